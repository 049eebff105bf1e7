"""GGUF v3 constants: metadata value types and ggml tensor types.

The reference never parses GGUF itself -- it hands models to LM Studio
(`/root/reference/nats_llm_studio.go:46-59`, `lms get`) whose llama.cpp engine
does. This framework loads GGUF directly, so the on-disk contract lives here.
"""
from __future__ import annotations

import enum

GGUF_MAGIC = b"GGUF"
GGUF_VERSION = 3
GGUF_DEFAULT_ALIGNMENT = 32
QK_K = 256


class GGUFValueType(enum.IntEnum):
    UINT8 = 0
    INT8 = 1
    UINT16 = 2
    INT16 = 3
    UINT32 = 4
    INT32 = 5
    FLOAT32 = 6
    BOOL = 7
    STRING = 8
    ARRAY = 9
    UINT64 = 10
    INT64 = 11
    FLOAT64 = 12


class GGMLType(enum.IntEnum):
    F32 = 0
    F16 = 1
    Q4_0 = 2
    Q4_1 = 3
    Q5_0 = 6
    Q5_1 = 7
    Q8_0 = 8
    Q8_1 = 9
    Q2_K = 10
    Q3_K = 11
    Q4_K = 12
    Q5_K = 13
    Q6_K = 14
    Q8_K = 15
    BF16 = 30


# (values per block, bytes per block)
GGML_BLOCK = {
    GGMLType.F32: (1, 4),
    GGMLType.F16: (1, 2),
    GGMLType.BF16: (1, 2),
    GGMLType.Q4_0: (32, 18),
    GGMLType.Q4_1: (32, 20),
    GGMLType.Q5_0: (32, 22),
    GGMLType.Q5_1: (32, 24),
    GGMLType.Q8_0: (32, 34),
    GGMLType.Q2_K: (256, 84),
    GGMLType.Q3_K: (256, 110),
    GGMLType.Q4_K: (256, 144),
    GGMLType.Q5_K: (256, 176),
    GGMLType.Q6_K: (256, 210),
}

# general.file_type (llama_ftype) values we emit / recognise.
FILE_TYPE_NAMES = {
    0: "F32",
    1: "F16",
    2: "Q4_0",
    3: "Q4_1",
    7: "Q8_0",
    8: "Q5_0",
    9: "Q5_1",
    10: "Q2_K",
    11: "Q3_K_S",
    12: "Q3_K_M",
    13: "Q3_K_L",
    15: "Q4_K_M",
    14: "Q4_K_S",
    17: "Q5_K_M",
    16: "Q5_K_S",
    18: "Q6_K",
    32: "BF16",
}
FILE_TYPE_IDS = {v: k for k, v in FILE_TYPE_NAMES.items()}


def tensor_nbytes(ggml_type: int, n_elements: int) -> int:
    blk, nbytes = GGML_BLOCK[GGMLType(ggml_type)]
    if n_elements % blk:
        raise ValueError(f"{GGMLType(ggml_type).name}: {n_elements} elements not a multiple of block {blk}")
    return n_elements // blk * nbytes
