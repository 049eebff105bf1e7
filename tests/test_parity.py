"""Parity pins that do NOT share code with the implementation under test (CPU).

* ggml block codecs: `gguf/quants.py` (the oracle of every GPU kernel test and of models/reference.py)
  against an independent element-by-element decoder written here from the ggml block definitions
  (get_scale_min_k4, the Q5_K high-bit masks, the Q6_K ql/qh/scale interleave), over
  random block bytes -- so 6-bit scales >= 16 (the high-bit path of get_scale_min_k4) and every
  nibble / high-bit combination are exercised -- plus hand-derived known-answer values.
* byte-level BPE: our tokenizer against HuggingFace `tokenizers` (installed offline) built from the
  SAME vocab + merges + pre-tokeniser regex, over a multilingual corpus. SentencePiece-BPE (Mixtral)
  parity stays unpinned: no sentencepiece model or reference file exists in the reference repo.
"""
import struct

import numpy as np
import pytest

from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.constants import GGMLType


def _h(b, off):
    return struct.unpack_from("<e", bytes(b[off:off + 2]))[0]


def _scale_min_k4(j, q):
    if j < 4:
        return q[j] & 63, q[j + 4] & 63
    return (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4), (q[j + 4] >> 4) | ((q[j] >> 6) << 4)


def spec_q4_k(b):
    d, dmin, sc, qs = _h(b, 0), _h(b, 2), list(b[4:16]), list(b[16:144])
    y = []
    for c in range(4):                      # 64-value chunks: low nibbles then high nibbles
        s1, m1 = _scale_min_k4(2 * c, sc)
        s2, m2 = _scale_min_k4(2 * c + 1, sc)
        q = qs[32 * c:32 * c + 32]
        y += [d * s1 * (v & 0xF) - dmin * m1 for v in q]
        y += [d * s2 * (v >> 4) - dmin * m2 for v in q]
    return y


def spec_q5_k(b):
    d, dmin, sc, qh, qs = _h(b, 0), _h(b, 2), list(b[4:16]), list(b[16:48]), list(b[48:176])
    y = []
    for c in range(4):
        s1, m1 = _scale_min_k4(2 * c, sc)
        s2, m2 = _scale_min_k4(2 * c + 1, sc)
        u1, u2 = 1 << (2 * c), 2 << (2 * c)
        q = qs[32 * c:32 * c + 32]
        y += [d * s1 * ((v & 0xF) + (16 if qh[l] & u1 else 0)) - dmin * m1 for l, v in enumerate(q)]
        y += [d * s2 * ((v >> 4) + (16 if qh[l] & u2 else 0)) - dmin * m2 for l, v in enumerate(q)]
    return y


def spec_q6_k(b):
    ql, qh = list(b[0:128]), list(b[128:192])
    sc = [v - 256 if v > 127 else v for v in b[192:208]]
    d = _h(b, 208)
    y = [0.0] * 256
    for n in range(2):
        L, H, S = ql[64 * n:64 * n + 64], qh[32 * n:32 * n + 32], sc[8 * n:8 * n + 8]
        for l in range(32):
            i = l // 16
            q1 = ((L[l] & 0xF) | (((H[l] >> 0) & 3) << 4)) - 32
            q2 = ((L[l + 32] & 0xF) | (((H[l] >> 2) & 3) << 4)) - 32
            q3 = ((L[l] >> 4) | (((H[l] >> 4) & 3) << 4)) - 32
            q4 = ((L[l + 32] >> 4) | (((H[l] >> 6) & 3) << 4)) - 32
            y[128 * n + l] = d * S[i] * q1
            y[128 * n + l + 32] = d * S[i + 2] * q2
            y[128 * n + l + 64] = d * S[i + 4] * q3
            y[128 * n + l + 96] = d * S[i + 6] * q4
    return y


def spec_q8_0(b):
    d = _h(b, 0)
    return [d * (v - 256 if v > 127 else v) for v in b[2:34]]


def _nib32(qs, j):
    """ggml 32-blocks: element j < 16 is the low nibble of qs[j], j >= 16 the high nibble of qs[j - 16]."""
    return (qs[j] & 0xF) if j < 16 else (qs[j - 16] >> 4)


def spec_q4_0(b):
    d = _h(b, 0)
    return [d * (_nib32(b[2:18], j) - 8) for j in range(32)]


def spec_q4_1(b):
    d, m = _h(b, 0), _h(b, 2)
    return [d * _nib32(b[4:20], j) + m for j in range(32)]


def spec_q5_0(b):
    d = _h(b, 0)
    qh = struct.unpack_from("<I", bytes(b[2:6]))[0]
    return [d * ((_nib32(b[6:22], j) | (((qh >> j) & 1) << 4)) - 16) for j in range(32)]


def spec_q5_1(b):
    d, m = _h(b, 0), _h(b, 2)
    qh = struct.unpack_from("<I", bytes(b[4:8]))[0]
    return [d * (_nib32(b[8:24], j) | (((qh >> j) & 1) << 4)) + m for j in range(32)]


def spec_q2_k(b):
    """ggml dequantize_row_q2_K: per 128-half, four 2-bit planes (shift 0, 2, 4, 6) of 32 bytes, each split
    into two 16-value sub-blocks with their own (scale, min) nibbles."""
    sc, qs = list(b[0:16]), list(b[16:80])
    d, dmin = _h(b, 80), _h(b, 82)
    y, k = [], 0
    for n in range(2):
        q = qs[32 * n:32 * n + 32]
        for j in range(4):
            for half in range(2):
                s = sc[k]
                k += 1
                y += [d * (s & 0xF) * ((q[16 * half + l] >> (2 * j)) & 3) - dmin * (s >> 4) for l in range(16)]
    return y


def spec_q3_k(b):
    """ggml dequantize_row_q3_K with the scale bytes decoded the way quantize_row_q3_K_reference packs
    them (low nibbles in bytes 0..7, top 2 bits in bytes 8..11) -- not the kmask word shuffle."""
    hm, qs, scb = list(b[0:32]), list(b[32:96]), list(b[96:108])
    d = _h(b, 108)
    scales = []
    for j in range(16):
        lo = (scb[j] & 0xF) if j < 8 else (scb[j - 8] >> 4)
        hi = (scb[8 + j % 4] >> (2 * (j // 4))) & 3
        scales.append((lo | (hi << 4)) - 32)
    y, k, m = [], 0, 1
    for n in range(2):
        q = qs[32 * n:32 * n + 32]
        for j in range(4):
            for half in range(2):
                dl = d * scales[k]
                k += 1
                for l in range(16):
                    v = (q[16 * half + l] >> (2 * j)) & 3
                    y.append(dl * (v - (0 if hm[16 * half + l] & m else 4)))
            m <<= 1
    return y


SPEC = {GGMLType.Q4_K: (144, 256, spec_q4_k), GGMLType.Q5_K: (176, 256, spec_q5_k),
        GGMLType.Q6_K: (210, 256, spec_q6_k), GGMLType.Q8_0: (34, 32, spec_q8_0),
        GGMLType.Q4_0: (18, 32, spec_q4_0), GGMLType.Q4_1: (20, 32, spec_q4_1),
        GGMLType.Q5_0: (22, 32, spec_q5_0), GGMLType.Q5_1: (24, 32, spec_q5_1),
        GGMLType.Q2_K: (84, 256, spec_q2_k), GGMLType.Q3_K: (110, 256, spec_q3_k)}


def _random_blocks(t, n, rng):
    size, _, _ = SPEC[t]
    raw = rng.integers(0, 256, size=(n, size), dtype=np.uint8)
    # finite f16 scale fields (random bytes could be NaN / inf): small normal values
    f16 = lambda: np.frombuffer(np.float16(rng.uniform(-0.05, 0.05)).tobytes(), np.uint8)
    for blk in raw:
        if t in (GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q4_1, GGMLType.Q5_1):
            blk[0:2], blk[2:4] = f16(), f16()
        elif t == GGMLType.Q6_K:
            blk[208:210] = f16()
        elif t == GGMLType.Q2_K:
            blk[80:82], blk[82:84] = f16(), f16()
        elif t == GGMLType.Q3_K:
            blk[108:110] = f16()
        else:
            blk[0:2] = f16()
    return raw


@pytest.mark.parametrize("t", [GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1, GGMLType.Q2_K,
                               GGMLType.Q3_K])
def test_quantizer_roundtrip_new_types(t):
    """The simple fits of gguf/quants.py produce blocks that decode (through the independent spec
    decoder) back to the input within the format's resolution."""
    rng = np.random.default_rng(100 + int(t))
    x = (rng.standard_normal(256 * 8) * 0.05).astype(np.float32)
    raw = Q.quantize(x, t)
    size, per, spec = SPEC[t]
    blocks = raw.reshape(-1, size)
    y = np.concatenate([np.array(spec([int(v) for v in b])) for b in blocks])
    tol = {GGMLType.Q2_K: 0.35, GGMLType.Q3_K: 0.3}.get(t, 0.12)
    assert np.abs(y - x).max() <= tol * np.abs(x).max(), np.abs(y - x).max()


@pytest.mark.parametrize("t", list(SPEC))
def test_codec_matches_independent_spec_decoder(t):
    rng = np.random.default_rng(int(t))
    size, per, spec = SPEC[t]
    raw = _random_blocks(t, 64, rng)
    got = Q.dequantize(raw.reshape(-1), t, (64 * per,)).reshape(64, per)
    want = np.array([spec([int(v) for v in b]) for b in raw], dtype=np.float64)
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-6 * np.abs(want).max())


def test_q4_k_known_answers_high_scale_bits():
    """get_scale_min_k4 sub-blocks 4..7 take their top 2 bits from bytes 0..7: hand-derived values."""
    b = np.zeros(144, np.uint8)
    b[0:2] = np.frombuffer(np.float16(2.0).tobytes(), np.uint8)     # d
    b[2:4] = np.frombuffer(np.float16(0.25).tobytes(), np.uint8)    # dmin
    sc = b[4:16]
    sc[0] = 0xC5     # sub-block 0: scale 5;  top bits 3 -> scale of sub-block 4
    sc[4] = 0x81     # sub-block 0: min 1;    top bits 2 -> min of sub-block 4
    sc[8] = 0x27     # sub-block 4: scale low 7 | 3 << 4 = 55, min low 2 | 2 << 4 = 34
    b[16 + 64] = 0x3F          # chunk 2 (sub-blocks 4, 5), l = 0: low nibble 15, high nibble 3
    b[16 + 0] = 0x09           # chunk 0 (sub-block 0), l = 0: low nibble 9
    y = Q.dequantize(b, GGMLType.Q4_K, (256,))
    assert y[0] == 2.0 * 5 * 9 - 0.25 * 1             # 89.75
    assert y[128] == 2.0 * 55 * 15 - 0.25 * 34        # 1641.5 (sub-block 4, 6-bit scale 55 >= 16)
    assert y[160] == 2.0 * 0 * 3 - 0.25 * 0           # sub-block 5: scale byte sc[9] = 0
    assert y[129] == -0.25 * 34


def test_q6_k_known_answers():
    b = np.zeros(210, np.uint8)
    b[208:210] = np.frombuffer(np.float16(0.5).tobytes(), np.uint8)
    b[192 + 0] = 3                     # scale of values 0..15
    b[192 + 6] = np.uint8(256 - 7)     # scale -7 of values 96..111 (q4 of the first half)
    b[0] = 0x5A                        # ql[0]: low 0xA (value 0), high 0x5 (value 64)
    b[128] = 0b11_00_10_01             # qh[0]: value 0 +1<<4, 32 +2<<4, 64 +0, 96 +3<<4
    b[32] = 0xF0                       # ql[32]: low 0 (value 32), high 0xF (value 96)
    y = Q.dequantize(b, GGMLType.Q6_K, (256,))
    assert y[0] == 0.5 * 3 * ((0xA | 16) - 32)         # -9.0
    assert y[96] == 0.5 * -7 * ((0xF | 48) - 32)       # -108.5
    assert y[32] == 0.5 * b[192 + 2] * ((0 | 32) - 32)  # scale 0 -> 0


# ---------------------------------------------------------------------------------------------
# tokenizer parity vs HuggingFace tokenizers
# ---------------------------------------------------------------------------------------------
CORPUS = [
    "Hello world! The quick brown fox jumps over the lazy dog.",
    "  leading spaces, trailing spaces   \n\n\tand tabs\r\n",
    "naïve café résumé Ångström straße",
    "Привет, как дела? Всё хорошо.",
    "東京は日本の首都です。中文测试，标点符号！",
    "مرحبا بالعالم", "नमस्ते दुनिया", "🙂😀👍🏽 emoji 🚀🚀",
    "def f(x):\n    return x ** 2  # comment\n",
    "numbers 1 12 123 1234 12345 3.14159 -42 1e-9",
    "It's I'm you're we've they'll she'd DON'T",
    "mixed CASE and under_score and camelCase and kebab-case",
    "''\"\"``((()))[[]]{{}}<<>>",
]


def _hf_bytelevel(tok, regex):
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers import Regex, models, pre_tokenizers
    vocab = {t: i for i, t in enumerate(tok.tokens)}
    merges = sorted(tok.ranks, key=tok.ranks.get)
    hf = tokenizers.Tokenizer(models.BPE(vocab=vocab, merges=merges, ignore_merges=False))
    hf.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(regex), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    return hf


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-qwen2", "tiny-granite"])
def test_bytelevel_bpe_matches_hf_tokenizers(tiny_models, name):
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.tokenizer import bpe
    tok = bpe.tokenizer_from_metadata(GGUFReader(tiny_models[name]).metadata)
    if not isinstance(tok, bpe.ByteLevelBPE):
        pytest.skip("not a byte-level BPE vocab")
    regex = tok.pretok.pattern
    hf = _hf_bytelevel(tok, regex)
    n_tok = 0
    for text in CORPUS:
        ours = tok.encode(text, add_bos=False, allow_special=False)
        theirs = hf.encode(text, add_special_tokens=False).ids
        assert ours == theirs, (name, text, ours[:20], theirs[:20])
        n_tok += len(ours)
    assert n_tok > 100
