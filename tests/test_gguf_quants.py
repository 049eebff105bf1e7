"""GGUF container + ggml block codec tests (CPU)."""
import numpy as np
import pytest

from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.constants import GGMLType
from nats_llm_studio_amd.gguf.reader import GGUFReader
from nats_llm_studio_amd.gguf.writer import GGUFWriter

TYPES = [GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.F16, GGMLType.BF16, GGMLType.F32]
TOL = {GGMLType.Q8_0: 0.02, GGMLType.Q4_K: 0.3, GGMLType.Q5_K: 0.15, GGMLType.Q6_K: 0.08,
       GGMLType.F16: 1e-3, GGMLType.BF16: 1e-2, GGMLType.F32: 0}


@pytest.mark.parametrize("t", TYPES)
def test_roundtrip(t):
    x = np.random.default_rng(0).standard_normal(256 * 8).astype(np.float32)
    raw = Q.quantize(x, t)
    y = Q.dequantize(raw, t, x.shape)
    assert np.abs(x - y).max() <= TOL[t] * max(1.0, np.abs(x).max()) + 1e-6


def test_block_sizes():
    x = np.zeros(512, np.float32)
    assert Q.quantize(x, GGMLType.Q4_K).size == 2 * 144
    assert Q.quantize(x, GGMLType.Q5_K).size == 2 * 176
    assert Q.quantize(x, GGMLType.Q6_K).size == 2 * 210
    assert Q.quantize(x, GGMLType.Q8_0).size == 16 * 34


def test_q4k_known_block():
    """Hand-built Q4_K block: d=1, dmin=0.5, sc_j = j+1, m_j = 2, q = index % 16."""
    sc = np.arange(1, 9, dtype=np.uint8)[None]
    m = np.full((1, 8), 2, np.uint8)
    blk = np.zeros(144, np.uint8)
    blk[0:2] = np.frombuffer(np.float16(1.0).tobytes(), np.uint8)
    blk[2:4] = np.frombuffer(np.float16(0.5).tobytes(), np.uint8)
    blk[4:16] = Q._pack_k4_scales(sc, m)[0]
    q = (np.arange(256) % 16).astype(np.uint8).reshape(4, 2, 32)
    blk[16:] = (q[:, 0] | (q[:, 1] << 4)).reshape(-1)
    y = Q.dequantize(blk, GGMLType.Q4_K, (256,))
    sub = np.arange(256) // 32
    expect = (sub + 1) * (np.arange(256) % 16) - 0.5 * 2
    np.testing.assert_allclose(y, expect)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0])
def test_random_blocks_stats(t):
    y = Q.dequantize(Q.random_blocks(t, 256 * 256, 0.02, np.random.default_rng(1)), t, (-1,))
    assert abs(y.mean()) < 0.005 and 0.01 < y.std() < 0.04


def test_gguf_roundtrip(tmp_path):
    p = str(tmp_path / "x.gguf")
    w = GGUFWriter(p, "llama")
    w.add("llama.block_count", 3)
    w.add("general.name", "unit")
    w.add("x.f", 1.5)
    w.add("x.flag", True)
    w.add("x.list", ["a", "bb", "ccc"])
    w.add("x.arr", np.arange(5, dtype=np.int32))
    a = np.random.default_rng(0).standard_normal((4, 256)).astype(np.float32)
    w.add_tensor("t.q4", (4, 256), GGMLType.Q4_K, Q.quantize(a, GGMLType.Q4_K))
    w.add_tensor("t.f32", (3,), GGMLType.F32, np.array([1, 2, 3], np.float32).view(np.uint8))
    w.write()
    r = GGUFReader(p)
    assert r.architecture == "llama" and r.get("llama.block_count") == 3
    assert r.get("x.list") == ["a", "bb", "ccc"] and r.get("x.flag") is True
    assert list(r.get("x.arr")) == [0, 1, 2, 3, 4] and abs(r.get("x.f") - 1.5) < 1e-6
    ti = r.tensor("t.q4")
    assert ti.np_shape == (4, 256) and ti.type_name == "Q4_K"
    assert (ti.offset % 32) == 0
    np.testing.assert_allclose(r.dequantized("t.f32"), [1, 2, 3])
    np.testing.assert_allclose(r.dequantized("t.q4"), Q.dequantize(Q.quantize(a, GGMLType.Q4_K), 12, (4, 256)))


def test_synthetic_model_plan(tiny_models):
    r = GGUFReader(tiny_models["tiny-llama"])
    assert r.file_type_name == "Q4_K_M"
    assert r.tensor("output.weight").type_name == "Q6_K"
    assert r.tensor("blk.0.attn_q.weight").type_name == "Q4_K"
    assert r.get("tokenizer.ggml.model") == "gpt2"


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0, GGMLType.F16,
                               GGMLType.F32])
def test_tiled_layout_is_a_permutation(t):
    """The tiled device layout keeps every byte (rows padded to 16 with zeros)."""
    import torch
    from nats_llm_studio_amd import ops
    rows, K = 37, 512
    raw = Q.random_blocks(t, rows * K, 0.05, np.random.default_rng(0))
    tl = ops.tile_layout(torch.from_numpy(raw.copy()), t, rows, K).numpy()
    rp = 48
    assert tl.size == rp // 16 * (K // 256) * ops.TILE_BYTES[t]
    assert sorted(tl.tolist()) == sorted(raw.tolist() + [0] * (tl.size - raw.size))


def test_prefill_blocks():
    from nats_llm_studio_amd.ops import PREFILL_QT as QT, prefill_blocks
    assert QT in (32, 64)            # attn_prefill: 64-token blocks (NLS_PREFILL_V1: 32)
    n0 = QT + QT // 4                # sequence 0 spans a full block and a partial one
    tseq = np.array([0] * n0 + [1] * 3 + [2] * 16)
    pos = np.concatenate([np.arange(n0), np.arange(50, 53), np.arange(16)])
    qb = prefill_blocks(tseq, pos, len(tseq))
    assert qb.tolist() == [[0, QT, 0, 0], [QT, n0 - QT, 0, QT], [n0, 3, 1, 50], [n0 + 3, 16, 2, 0]]
