"""Tokenizers driven purely by GGUF metadata (`tokenizer.ggml.*`).

* `ByteLevelBPE`  -- tokenizer.ggml.model == "gpt2" (Llama-3, Granite): GPT-2
  byte->unicode alphabet, regex pre-tokeniser, rank-ordered merges.
* `SentencePieceBPE` -- tokenizer.ggml.model == "llama" (Mixtral / Llama-2):
  score-ordered merges over "▁"-normalised text with <0xXX> byte fallback.

In the reference all of this happens inside LM Studio behind
`POST /api/v0/chat/completions` (`/root/reference/nats_llm_studio.go:158-179`).
"""
from __future__ import annotations

import functools
import heapq
from typing import Dict, List, Optional, Sequence

import regex as re

try:    # native merge loops (csrc/tokcore, GIL released); the pure-Python loops below are the reference
    from . import _tokcore
except ImportError:          # not built (python -m nats_llm_studio_amd.build)
    _tokcore = None

# Llama-3 pre-tokeniser (llama.cpp LLAMA_VOCAB_PRE_TYPE_LLAMA3)
LLAMA3_PRETOK = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                 r"|\s*[\r\n]+|\s+(?!\S)|\s+")
# Qwen2 pre-tokeniser (llama.cpp LLAMA_VOCAB_PRE_TYPE_QWEN2): single digits
QWEN2_PRETOK = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                r"|\s*[\r\n]+|\s+(?!\S)|\s+")
GPT2_PRETOK = r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"

TOKEN_TYPE_NORMAL = 1
TOKEN_TYPE_UNKNOWN = 2
TOKEN_TYPE_CONTROL = 3
TOKEN_TYPE_USER_DEFINED = 4
TOKEN_TYPE_UNUSED = 5
TOKEN_TYPE_BYTE = 6


@functools.lru_cache(maxsize=1)
def bytes_to_unicode() -> Dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


class _Base:
    def __init__(self, tokens: Sequence[str], token_types: Optional[Sequence[int]], bos_id: Optional[int],
                 eos_id: Optional[int], add_bos: bool):
        self.tokens = list(tokens)
        self.vocab = {t: i for i, t in enumerate(self.tokens)}
        self.token_types = list(token_types) if token_types is not None else [TOKEN_TYPE_NORMAL] * len(self.tokens)
        self.bos_id = bos_id
        self.eos_id = eos_id
        self.add_bos = add_bos
        # special (control / user-defined) tokens are matched verbatim before BPE
        self.special = {t: i for i, t in enumerate(self.tokens)
                        if self.token_types[i] in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_USER_DEFINED)}
        if self.special:
            pat = "|".join(re.escape(s) for s in sorted(self.special, key=len, reverse=True))
            self._special_re = re.compile(f"({pat})")
        else:
            self._special_re = None

    @property
    def n_vocab(self) -> int:
        return len(self.tokens)

    def _split_special(self, text: str, allow_special: bool):
        if not allow_special or self._special_re is None:
            return [(text, False)]
        out = []
        for part in self._special_re.split(text):
            if not part:
                continue
            out.append((part, part in self.special))
        return out

    def encode(self, text: str, add_bos: Optional[bool] = None, allow_special: bool = True) -> List[int]:
        ids: List[int] = []
        if (self.add_bos if add_bos is None else add_bos) and self.bos_id is not None:
            ids.append(self.bos_id)
        for part, is_special in self._split_special(text, allow_special):
            if is_special:
                ids.append(self.special[part])
            else:
                ids.extend(self._encode_plain(part))
        return ids

    def is_control(self, tid: int) -> bool:
        return 0 <= tid < len(self.token_types) and self.token_types[tid] == TOKEN_TYPE_CONTROL


class ByteLevelBPE(_Base):
    def __init__(self, tokens, merges: Sequence[str], token_types=None, bos_id=None, eos_id=None,
                 add_bos: bool = True, pre: str = "llama-bpe"):
        super().__init__(tokens, token_types, bos_id, eos_id, add_bos)
        self.ranks = {}
        for i, m in enumerate(merges):
            a, _, b = m.partition(" ")
            self.ranks[(a, b)] = i
        self.b2u = bytes_to_unicode()
        self.u2b = {v: k for k, v in self.b2u.items()}
        self.pretok = re.compile(GPT2_PRETOK if pre in ("gpt2", "default") else
                                 QWEN2_PRETOK if pre == "qwen2" else LLAMA3_PRETOK)
        # the same pattern in the native pre-tokeniser (csrc/tokcore Pretok: 0 llama3, 1 qwen2, 2 gpt2)
        self.pre_mode = 2 if pre in ("gpt2", "default") else 1 if pre == "qwen2" else 0
        self._cache: Dict[str, List[int]] = {}
        self.native = self._native_core()

    def _native_core(self):
        """The C++ merge loop when every byte has its own token and every merge's result is a vocabulary
        entry (true of real BPE vocabularies; otherwise the Python loop, whose fallback splits unknown
        symbols into bytes, stays in charge)."""
        if _tokcore is None:
            return None
        byte_ids = [self.vocab.get(self.b2u[b]) for b in range(256)]
        if any(i is None for i in byte_ids):
            return None
        merges = []
        for (a, b), _ in sorted(self.ranks.items(), key=lambda kv: kv[1]):
            ia, ib, im = self.vocab.get(a), self.vocab.get(b), self.vocab.get(a + b)
            if ia is None or ib is None or im is None:
                return None
            merges.append((ia, ib, im))
        return _tokcore.ByteLevel(byte_ids, merges)

    def _bpe(self, word: str) -> List[str]:
        parts = list(word)
        if len(parts) < 2:
            return parts
        while True:
            best = None
            best_rank = None
            for i in range(len(parts) - 1):
                r = self.ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = i, r
            if best is None:
                return parts
            parts = parts[:best] + [parts[best] + parts[best + 1]] + parts[best + 2:]

    def _encode_plain(self, text: str) -> List[int]:
        if self.native is not None:
            if hasattr(self.native, "encode_text"):
                # pre-tokeniser + merges natively, the GIL released for the whole text: a burst of requests
                # tokenises in parallel on the handler threads
                return self.native.encode_text(text, self.pre_mode)
            return self.native.encode_pieces([p.encode("utf-8") for p in self.pretok.findall(text, concurrent=True)])
        return self._encode_plain_py(text)

    def _encode_plain_py(self, text: str) -> List[int]:
        out: List[int] = []
        for piece in self.pretok.findall(text):
            hit = self._cache.get(piece)
            if hit is None:
                u = "".join(self.b2u[b] for b in piece.encode("utf-8"))
                hit = []
                for sym in self._bpe(u):
                    tid = self.vocab.get(sym)
                    if tid is None:            # unmergeable: fall back to single byte symbols
                        hit.extend(self.vocab[c] for c in sym)
                    else:
                        hit.append(tid)
                if len(self._cache) < 65536:
                    self._cache[piece] = hit
            out.extend(hit)
        return out

    def token_bytes(self, tid: int) -> bytes:
        t = self.tokens[tid]
        if self.token_types[tid] in (TOKEN_TYPE_CONTROL, TOKEN_TYPE_USER_DEFINED):
            return t.encode("utf-8")
        try:
            return bytes(self.u2b[c] for c in t)
        except KeyError:
            return t.encode("utf-8")

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        buf = bytearray()
        for i in ids:
            if skip_special and self.is_control(i):
                continue
            buf += self.token_bytes(i)
        return buf.decode("utf-8", errors="replace")


class SentencePieceBPE(_Base):
    SPACE = "▁"

    def __init__(self, tokens, scores: Sequence[float], token_types=None, bos_id=1, eos_id=2,
                 add_bos: bool = True, add_space_prefix: bool = True):
        super().__init__(tokens, token_types, bos_id, eos_id, add_bos)
        self.scores = list(scores)
        self.add_space_prefix = add_space_prefix
        self.byte_ids = {}
        for i, t in enumerate(self.tokens):
            if self.token_types[i] == TOKEN_TYPE_BYTE and len(t) == 6 and t.startswith("<0x"):
                self.byte_ids[int(t[3:5], 16)] = i
        self.native = (_tokcore.Spm(self.tokens, [float(x) for x in self.scores],
                                    [self.byte_ids.get(b, -1) for b in range(256)]) if _tokcore is not None else None)

    def _encode_plain(self, text: str) -> List[int]:
        if not text:
            return []
        s = text.replace(" ", self.SPACE)
        if self.add_space_prefix:
            s = self.SPACE + s
        if self.native is not None:
            return self.native.encode(s)
        return self._merge_py(s)

    def _merge_py(self, s: str) -> List[int]:
        # symbols as a doubly linked list; merge best-scoring pair first
        sym = list(s)
        prev = list(range(-1, len(sym) - 1))
        nxt = list(range(1, len(sym) + 1))
        nxt[-1] = -1
        alive = [True] * len(sym)
        heap = []

        def push(i):
            j = nxt[i]
            if j < 0:
                return
            tid = self.vocab.get(sym[i] + sym[j])
            if tid is not None:
                heapq.heappush(heap, (-self.scores[tid], i, sym[i], sym[j]))

        for i in range(len(sym) - 1):
            push(i)
        while heap:
            _, i, a, b = heapq.heappop(heap)
            j = nxt[i] if alive[i] else -1
            if j < 0 or not alive[j] or sym[i] != a or sym[j] != b:
                continue
            sym[i] = a + b
            alive[j] = False
            nxt[i] = nxt[j]
            if nxt[j] >= 0:
                prev[nxt[j]] = i
            if prev[i] >= 0:
                push(prev[i])
            push(i)
        out: List[int] = []
        i = 0
        while i >= 0 and i < len(sym):
            if alive[i]:
                tid = self.vocab.get(sym[i])
                if tid is not None:
                    out.append(tid)
                else:
                    for b in sym[i].encode("utf-8"):
                        out.append(self.byte_ids.get(b, 0))
            i = nxt[i]
        return out

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        buf = bytearray()
        for i in ids:
            if skip_special and self.is_control(i):
                continue
            tt = self.token_types[i]
            t = self.tokens[i]
            if tt == TOKEN_TYPE_BYTE and t.startswith("<0x"):
                buf.append(int(t[3:5], 16))
            else:
                buf += t.replace(self.SPACE, " ").encode("utf-8")
        out = buf.decode("utf-8", errors="replace")
        if self.add_space_prefix and out.startswith(" "):
            out = out[1:]
        return out


def tokenizer_from_metadata(md: dict):
    model = md.get("tokenizer.ggml.model", "gpt2")
    tokens = md["tokenizer.ggml.tokens"]
    ttypes = md.get("tokenizer.ggml.token_type")
    ttypes = [int(x) for x in ttypes] if ttypes is not None else None
    bos = md.get("tokenizer.ggml.bos_token_id")
    eos = md.get("tokenizer.ggml.eos_token_id")
    add_bos = bool(md.get("tokenizer.ggml.add_bos_token", True))
    if model == "gpt2":
        return ByteLevelBPE(tokens, md.get("tokenizer.ggml.merges", []), ttypes,
                            None if bos is None else int(bos), None if eos is None else int(eos),
                            add_bos, md.get("tokenizer.ggml.pre", "llama-bpe"))
    if model == "llama":
        scores = md.get("tokenizer.ggml.scores")
        scores = [float(x) for x in scores] if scores is not None else [0.0] * len(tokens)
        return SentencePieceBPE(tokens, scores, ttypes, None if bos is None else int(bos),
                                None if eos is None else int(eos), add_bos,
                                bool(md.get("tokenizer.ggml.add_space_prefix", True)))
    raise NotImplementedError(f"tokenizer model {model!r}")


class StreamDecoder:
    """Incremental detokenisation for streamed deltas (`stream: true`).

    Decoding one token at a time splits multi-byte UTF-8 characters (a CJK character or an emoji
    is often 2-4 byte-level tokens) and drops SentencePiece word-boundary spaces. This keeps a
    short window: `prefix` = text of ids[p:r] already emitted, `full` = text of ids[p:]; the delta
    is what `full` adds, held back while it still ends in an incomplete sequence (U+FFFD)."""

    def __init__(self, tok):
        self.tok = tok
        self.ids = []
        self.p = 0      # window start
        self.r = 0      # end of the already-emitted part of the window

    def push(self, t: int) -> str:
        self.ids.append(int(t))
        prefix = self.tok.decode(self.ids[self.p:self.r]) if self.r > self.p else ""
        full = self.tok.decode(self.ids[self.p:])
        if full.endswith("�") or len(full) <= len(prefix):
            return ""
        delta = full[len(prefix):]
        self.p, self.r = self.r, len(self.ids)
        return delta
