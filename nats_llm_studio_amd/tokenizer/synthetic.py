"""Deterministic synthetic vocabularies for random-init checkpoints.

No real tokenizer files can be fetched (no network), so synthetic GGUFs carry a
small BPE trained here on an embedded corpus, padded with reserved special
tokens up to the real model's vocab size (the way Llama-3 pads its own vocab),
so the embedding / lm_head shapes are exactly the north-star shapes.
"""
from __future__ import annotations

from collections import Counter
from typing import List, Tuple

import regex as re

from .bpe import (LLAMA3_PRETOK, TOKEN_TYPE_BYTE, TOKEN_TYPE_CONTROL, TOKEN_TYPE_NORMAL,
                  TOKEN_TYPE_UNUSED, bytes_to_unicode)

CORPUS = """
The quick brown fox jumps over the lazy dog. A language model predicts the next token given the
previous tokens. Messages arrive over NATS request reply subjects and the worker answers with a JSON
envelope. The model runs on the GPU with quantized weights, paged key value caches and fused kernels.
Hello! How are you today? I am fine, thank you. What is the capital of France? The capital of France
is Paris. Please write a short poem about the sea. The sea is wide and deep and blue, it sings a song
for me and you. Tell me a story about a robot who learns to paint. Once upon a time there was a robot
named Ada who lived in a quiet town. Every morning she watched the sun rise over the hills and wished
she could capture its colors. Numbers like 1, 2, 3, 42, 100 and 2024 appear in text too. Code such as
def main(): return 0 or for i in range(10): print(i) is common. You are a helpful assistant. The user
asks a question and the assistant answers it clearly and concisely. Throughput, latency, tokens per
second, and memory bandwidth matter for inference servers. Matrix multiplication on matrix cores.
"""

LLAMA3_SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|reserved_special_token_0|>",
                   "<|reserved_special_token_1|>", "<|finetune_right_pad_id|>", "<|step_id|>",
                   "<|start_header_id|>", "<|end_header_id|>", "<|eom_id|>", "<|eot_id|>", "<|python_tag|>"]

LLAMA3_TEMPLATE = (
    "{{- bos_token }}"
    "{%- for message in messages %}"
    "{{- '<|start_header_id|>' + message['role'] + '<|end_header_id|>\\n\\n' + message['content'] | trim + '<|eot_id|>' }}"
    "{%- endfor %}"
    "{%- if add_generation_prompt %}{{- '<|start_header_id|>assistant<|end_header_id|>\\n\\n' }}{%- endif %}"
)

GRANITE_TEMPLATE = (
    "{%- for message in messages %}"
    "{{- '<|start_of_role|>' + message['role'] + '<|end_of_role|>' + message['content'] + '<|end_of_text|>\\n' }}"
    "{%- endfor %}"
    "{%- if add_generation_prompt %}{{- '<|start_of_role|>assistant<|end_of_role|>' }}{%- endif %}"
)

MISTRAL_TEMPLATE = (
    "{{- bos_token }}"
    "{%- for message in messages %}"
    "{%- if message['role'] == 'user' %}{{- '[INST] ' + message['content'] + ' [/INST]' }}"
    "{%- elif message['role'] == 'system' %}{{- '[INST] ' + message['content'] + ' [/INST]' }}"
    "{%- else %}{{- message['content'] + eos_token }}{%- endif %}"
    "{%- endfor %}"
)


def _train_bytelevel_merges(n_merges: int) -> List[Tuple[str, str]]:
    b2u = bytes_to_unicode()
    pre = re.compile(LLAMA3_PRETOK)
    words = Counter("".join(b2u[b] for b in w.encode()) for w in pre.findall(CORPUS))
    seqs = {w: list(w) for w in words}
    merges = []
    for _ in range(n_merges):
        pairs = Counter()
        for w, c in words.items():
            s = seqs[w]
            for i in range(len(s) - 1):
                pairs[(s[i], s[i + 1])] += c
        if not pairs:
            break
        (a, b), cnt = max(pairs.items(), key=lambda kv: (kv[1], kv[0]))
        if cnt < 2:
            break
        merges.append((a, b))
        for w in seqs:
            s = seqs[w]
            i, out = 0, []
            while i < len(s):
                if i + 1 < len(s) and s[i] == a and s[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(s[i])
                    i += 1
            seqs[w] = out
    return merges


def bytelevel_vocab(n_vocab: int, specials=None, n_merges: int = 400):
    """-> tokens, token_types, merges (gguf strings), special ids dict."""
    specials = list(specials if specials is not None else LLAMA3_SPECIALS)
    b2u = bytes_to_unicode()
    tokens = [b2u[b] for b in range(256)]
    types = [TOKEN_TYPE_NORMAL] * 256
    merges = _train_bytelevel_merges(n_merges)
    for a, b in merges:
        if a + b not in tokens:
            tokens.append(a + b)
            types.append(TOKEN_TYPE_NORMAL)
    n_regular = n_vocab - len(specials)
    if len(tokens) > n_regular:
        raise ValueError("vocab too small for synthetic BPE")
    k = 0
    while len(tokens) < n_regular:          # pad regular range with unused placeholders
        tokens.append(f"<|unused_{k}|>")
        types.append(TOKEN_TYPE_UNUSED)
        k += 1
    ids = {}
    for s in specials:
        ids[s] = len(tokens)
        tokens.append(s)
        types.append(TOKEN_TYPE_CONTROL)
    return tokens, types, [f"{a} {b}" for a, b in merges], ids


def spm_vocab(n_vocab: int, n_merges: int = 400):
    """Llama-2/Mistral-style SentencePiece vocab: <unk>, <s>, </s>, 256 byte tokens, merged pieces."""
    tokens = ["<unk>", "<s>", "</s>"]
    types = [2, TOKEN_TYPE_CONTROL, TOKEN_TYPE_CONTROL]
    scores = [0.0, 0.0, 0.0]
    for b in range(256):
        tokens.append(f"<0x{b:02X}>")
        types.append(TOKEN_TYPE_BYTE)
        scores.append(0.0)
    text = CORPUS.replace("\n", " ")
    words = Counter(("▁" + w) for w in text.split())
    chars = sorted({c for w in words for c in w})
    for c in chars:
        tokens.append(c)
        types.append(TOKEN_TYPE_NORMAL)
        scores.append(-1000.0)
    seqs = {w: list(w) for w in words}
    score = -1.0
    for _ in range(n_merges):
        pairs = Counter()
        for w, c in words.items():
            s = seqs[w]
            for i in range(len(s) - 1):
                pairs[(s[i], s[i + 1])] += c
        if not pairs:
            break
        (a, b), cnt = max(pairs.items(), key=lambda kv: (kv[1], kv[0]))
        if cnt < 2 or len(tokens) >= n_vocab:
            break
        if a + b not in tokens:
            tokens.append(a + b)
            types.append(TOKEN_TYPE_NORMAL)
            scores.append(score)
            score -= 1.0
        for w in seqs:
            s = seqs[w]
            i, out = 0, []
            while i < len(s):
                if i + 1 < len(s) and s[i] == a and s[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(s[i])
                    i += 1
            seqs[w] = out
    k = 0
    while len(tokens) < n_vocab:
        tokens.append(f"<unused{k}>")
        types.append(TOKEN_TYPE_UNUSED)
        scores.append(-1e9)
        k += 1
    return tokens[:n_vocab], types[:n_vocab], scores[:n_vocab]


# Qwen2 / ChatML
QWEN2_SPECIALS = ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]
CHATML_TEMPLATE = (
    "{% for message in messages %}"
    "{% if loop.first and message['role'] != 'system' %}<|im_start|>system\nYou are a helpful assistant.<|im_end|>\n{% endif %}"
    "<|im_start|>{{ message['role'] }}\n{{ message['content'] }}<|im_end|>\n"
    "{% endfor %}"
    "{% if add_generation_prompt %}<|im_start|>assistant\n{% endif %}"
)
