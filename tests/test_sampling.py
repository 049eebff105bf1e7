"""CPU sampler reference: counter-based variates and inverse-CDF draws in index order (the
semantics of csrc/kernels/sample.hip, so seeded requests agree across sampling paths)."""
import torch

from nats_llm_studio_amd.engine.sampling import SamplingParams, sample_rows, uniform01


def test_uniform01_is_a_pure_function_of_seed_and_position():
    a = [uniform01(7, p) for p in range(100)]
    assert a == [uniform01(7, p) for p in range(100)]
    assert a != [uniform01(8, p) for p in range(100)]
    assert all(0.0 <= u < 1.0 for u in a)
    assert abs(sum(a) / len(a) - 0.5) < 0.1
    # 24-bit mantissa: exactly representable in fp32 (the kernel's float)
    assert all(float(torch.tensor(u, dtype=torch.float32)) == u for u in a)


def test_inverse_cdf_draw_in_index_order():
    lg = torch.log(torch.tensor([[0.1, 0.2, 0.3, 0.4]]))
    p = SamplingParams(temperature=1.0)
    # cumulative masses 0.1 0.3 0.6 1.0: u picks the first index whose cdf exceeds u
    for u, want in ((0.05, 0), (0.15, 1), (0.29, 1), (0.31, 2), (0.65, 3), (0.999, 3)):
        assert sample_rows(lg.clone(), [p], [[]], [u]) == [want]
    # top_k=2 keeps indices 2, 3 (mass 0.3, 0.4 of 0.7)
    pk = SamplingParams(temperature=1.0, top_k=2)
    assert sample_rows(lg.clone(), [pk], [[]], [0.0]) == [2]
    assert sample_rows(lg.clone(), [pk], [[]], [0.5]) == [3]
    # top_p=0.5 keeps the top set reaching half the mass: {3, 2}
    pp = SamplingParams(temperature=1.0, top_p=0.5)
    assert sample_rows(lg.clone(), [pp], [[]], [0.1]) == [2]


def test_masked_logits_and_seeded_reproducibility():
    torch.manual_seed(0)
    lg = torch.randn(1, 1000)
    lg[0, ::2] = float("-inf")
    p = SamplingParams(temperature=0.8, top_k=5, top_p=0.9)
    toks = [sample_rows(lg.clone(), [p], [[]], [uniform01(42, i)])[0] for i in range(50)]
    assert toks == [sample_rows(lg.clone(), [p], [[]], [uniform01(42, i)])[0] for i in range(50)]
    top5 = set(torch.topk(lg[0], 5).indices.tolist())
    assert set(toks) <= top5 and all(t % 2 == 1 for t in toks)


def test_omitted_fields_follow_the_documented_profile(monkeypatch):
    """Parity unpinned (no reference fixture): omitted sampling fields of a SAMPLING request take LM Studio's
    preset (top-k 40, top-p 0.95, min-p 0.05, repeat penalty 1.1); omitted / zero temperature stays greedy;
    explicit fields always win; NLS_SAMPLING_DEFAULTS selects lmstudio-full / neutral."""
    from nats_llm_studio_amd.engine.sampling import SamplingParams as S
    monkeypatch.delenv("NLS_SAMPLING_DEFAULTS", raising=False)
    p = S.from_request({"model": "m", "temperature": 0.7})          # the reference README's payload
    assert (p.temperature, p.top_k, p.top_p, p.min_p, p.repeat_penalty) == (0.7, 40, 0.95, 0.05, 1.1)
    assert S.from_request({"model": "m"}).greedy and S.from_request({"temperature": 0}).greedy
    p = S.from_request({"temperature": 0.9, "top_k": 0, "top_p": 1.0, "min_p": 0, "repeat_penalty": 1.0})
    assert (p.top_k, p.top_p, p.min_p, p.repeat_penalty) == (0, 1.0, 0.0, 1.0)
    # repeat_penalty 0 ("off" for some clients) or negative is the neutral 1.0, never a division by zero
    for rp in (0, 0.0, -1.5):
        p = S.from_request({"temperature": 0.7, "repeat_penalty": rp})
        assert p.repeat_penalty == 1.0
    assert S.from_request({"repeat_penalty": 0}).greedy
    monkeypatch.setenv("NLS_SAMPLING_DEFAULTS", "lmstudio-full")
    p = S.from_request({"model": "m"})
    assert (p.temperature, p.top_k, p.repeat_penalty) == (0.8, 40, 1.1) and not p.greedy
    monkeypatch.setenv("NLS_SAMPLING_DEFAULTS", "neutral")
    p = S.from_request({"temperature": 0.7})
    assert (p.top_k, p.top_p, p.min_p, p.repeat_penalty) == (0, 1.0, 0.0, 1.0)
