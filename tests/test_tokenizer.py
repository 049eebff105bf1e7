"""Tokenizer + chat template from GGUF metadata (CPU)."""
import pytest

from nats_llm_studio_amd.gguf.reader import GGUFReader
from nats_llm_studio_amd.tokenizer.bpe import tokenizer_from_metadata
from nats_llm_studio_amd.tokenizer.chat_template import ChatTemplate

TEXTS = ["Hello world!", "The capital of France is Paris.", "  spaces  and\nnewlines\n\n", "naïve café 😀",
         "def main(): return 42", ""]


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-granite", "tiny-qwen2"])
def test_roundtrip(tiny_models, name):
    md = GGUFReader(tiny_models[name]).metadata
    tok = tokenizer_from_metadata(md)
    for t in TEXTS:
        ids = tok.encode(t, add_bos=False)
        assert tok.decode(ids) == t, (name, t, ids)


def test_special_tokens_and_template(tiny_models):
    md = GGUFReader(tiny_models["tiny-llama"]).metadata
    tok = tokenizer_from_metadata(md)
    ct = ChatTemplate(md["tokenizer.chat_template"], tok.tokens[tok.bos_id])
    s = ct.render([{"role": "system", "content": "Be brief."}, {"role": "user", "content": "Hi"}])
    assert s.startswith("<|begin_of_text|><|start_header_id|>system<|end_header_id|>")
    assert s.endswith("<|start_header_id|>assistant<|end_header_id|>\n\n")
    ids = tok.encode(s, add_bos=False)
    assert ids[0] == tok.bos_id
    assert tok.vocab["<|eot_id|>"] in ids
    assert tok.decode(ids, skip_special=False) == s


def test_bpe_merges_applied(tiny_models):
    md = GGUFReader(tiny_models["tiny-llama"]).metadata
    tok = tokenizer_from_metadata(md)
    ids = tok.encode("the the the", add_bos=False)
    assert len(ids) < len("the the the")


def test_multipart_content(tiny_models):
    md = GGUFReader(tiny_models["tiny-granite"]).metadata
    ct = ChatTemplate(md["tokenizer.chat_template"])
    s = ct.render([{"role": "user", "content": [{"type": "text", "text": "a"}, {"type": "text", "text": "b"}]}])
    assert "<|start_of_role|>user<|end_of_role|>ab" in s


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-granite", "tiny-qwen2"])
def test_stream_decoder_reassembles_text(tiny_models, name):
    """Streamed deltas concatenate to the full decode: multi-byte UTF-8 split over byte tokens is held
    back until complete, SentencePiece word spaces survive token-by-token emission."""
    from nats_llm_studio_amd.tokenizer.bpe import StreamDecoder
    tok = tokenizer_from_metadata(GGUFReader(tiny_models[name]).metadata)
    for t in TEXTS:
        ids = tok.encode(t, add_bos=False)
        sd = StreamDecoder(tok)
        deltas = [sd.push(i) for i in ids]
        assert "".join(deltas) == tok.decode(ids), (name, t, deltas)
        assert all("�" not in d for d in deltas)


def test_qwen2_chatml_and_single_digit_pretokeniser(tiny_models):
    md = GGUFReader(tiny_models["tiny-qwen2"]).metadata
    tok = tokenizer_from_metadata(md)
    ct = ChatTemplate(md["tokenizer.chat_template"])
    s = ct.render([{"role": "user", "content": "Hi"}])
    assert s.startswith("<|im_start|>system\n") and s.endswith("<|im_start|>assistant\n")
    assert tok.tokens[tok.eos_id] == "<|im_end|>"
    assert [p for p in tok.pretok.findall("x 2024")] == ["x", " ", "2", "0", "2", "4"]


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-qwen2", "tiny-granite"])
def test_native_merge_loop_matches_python(tiny_models, name):
    """csrc/tokcore (C++ merge loops, GIL released) gives exactly the Python reference's ids."""
    import random
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.tokenizer.bpe import tokenizer_from_metadata
    tok = tokenizer_from_metadata(GGUFReader(tiny_models[name]).metadata)
    assert tok.native is not None, "native tokenizer core not built"
    rnd = random.Random(7)
    alphabet = list("abcdefghijklmnopqrstuvwxyz ABCXYZ0123456789  \n\t.,;:!?'\"-()") + \
        ["é", "ü", "中", "文", "😀", "ß", "  ", "\n\n", "'s", "'ll", "12345", "hello", " world"]
    texts = ["", "a", "hello world", "The quick brown fox jumps over the lazy dog 1234567 times!"]
    texts += ["".join(rnd.choice(alphabet) for _ in range(rnd.randint(1, 200))) for _ in range(150)]
    for t in texts:
        nat = tok.encode(t, add_bos=False)
        keep, tok.native = tok.native, None
        try:
            ref = tok.encode(t, add_bos=False)
        finally:
            tok.native = keep
        assert nat == ref, (t, nat, ref)


def test_spm_duplicate_token_strings_native_matches_python():
    """A vocabulary that holds the same string twice (seen in converted GGUFs): the native SentencePiece core
    keeps the LAST id, like the Python reference's {t: i} map and llama.cpp's token_to_id."""
    from nats_llm_studio_amd.tokenizer import bpe
    if bpe._tokcore is None:
        pytest.skip("native tokenizer core not built")
    toks = ["<unk>", "<s>", "</s>"] + [f"<0x{b:02X}>" for b in range(256)] + \
        ["▁", "a", "b", "ab", "▁a", "ab", "▁ab", "b", "▁b", "ba"]
    types = [bpe.TOKEN_TYPE_UNKNOWN, bpe.TOKEN_TYPE_CONTROL, bpe.TOKEN_TYPE_CONTROL] + \
        [bpe.TOKEN_TYPE_BYTE] * 256 + [bpe.TOKEN_TYPE_NORMAL] * 10
    scores = [0.0] * 259 + [-1.0, -2.0, -2.5, -0.5, -0.7, -0.4, -0.3, -2.2, -0.9, -1.5]
    tok = bpe.SentencePieceBPE(toks, scores, types)
    assert tok.native is not None
    for t in ["ab", "a b", "abab ba", "bab", "b a ab ba ab", "xyz ab", "ababababab"]:
        nat = tok.encode(t, add_bos=False)
        keep, tok.native = tok.native, None
        try:
            ref = tok.encode(t, add_bos=False)
        finally:
            tok.native = keep
        assert nat == ref, (t, nat, ref)
    assert tok.encode("ab", add_bos=False) == [259 + 6]          # "▁ab": the only id of that string
    assert tok.encode("bab", add_bos=False) == [259 + 8, 259 + 5]  # "▁b" + the duplicate "ab": its LAST id


def test_native_pretokenizer_matches_regex():
    """csrc/tokcore's hand-written pre-tokenisers (llama3 / qwen2 / gpt2) split random texts exactly as the regex
    module does with bpe.py's patterns: letters, digits, Unicode whitespace, CR/LF runs, contractions in both
    cases (and U+017F, which case-folds to 's'), combining marks, CJK, emoji, punctuation runs."""
    import random

    import regex

    from nats_llm_studio_amd.tokenizer import bpe
    tc = pytest.importorskip("nats_llm_studio_amd.tokenizer._tokcore")
    alphabet = (list("abcXYZ sStTrReEvVmMlLdD'") + list("0123456789") + [" ", " ", "  ", "\n", "\r", "\t", "\r\n"]
                + list("!?.,;:-_()[]{}\"'`~@#$%^&*+=/\\|<>") + ["é", "ß", "Ω", "ж", "ſ", "ǅ", "́", "̀",
                "中", "文", "日本", "한", "😀", "👍🏽", "٣", "Ⅻ", "½", "²", " ", " ", "　", " ",
                "\u0085", "\x0b", "\x0c", "\x1c", "​", "﻿", "'S", "'LL", "'Re", "'ve", "'D", "'ſ"])
    rng = random.Random(5)
    pats = {0: bpe.LLAMA3_PRETOK, 1: bpe.QWEN2_PRETOK, 2: bpe.GPT2_PRETOK}
    for mode, pat in pats.items():
        rx = regex.compile(pat)
        for _ in range(3000):
            text = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 40)))
            want = [p.encode("utf-8") for p in rx.findall(text)]
            got = tc.pretokenize(text.encode("utf-8").decode("utf-8"), mode)
            assert got == want, (mode, text, got, want)
