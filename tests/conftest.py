import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP kernel library")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def tiny_models(tmp_path_factory):
    """Synthetic tiny GGUFs of each supported family (written once per session)."""
    from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
    d = tmp_path_factory.mktemp("models")
    out = {}
    for name in ("tiny-llama", "tiny-mixtral", "tiny-granite", "tiny-llama31", "tiny-qwen2"):
        p = str(d / f"{name}.gguf")
        write_synthetic_gguf(p, name, "Q4_K_M", seed=0)
        out[name] = p
    return out


NEW_FTYPES = ("Q4_0", "Q4_1", "Q5_0", "Q5_1", "Q3_K_M", "Q2_K")


@pytest.fixture(scope="session")
def tiny_ftypes(tmp_path_factory):
    """tiny-llama written in every GGUF mix that is re-encoded at load (ops/transcode.py)."""
    from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
    d = tmp_path_factory.mktemp("ftypes")
    out = {}
    for ft in NEW_FTYPES:
        p = str(d / f"tiny-llama-{ft}.gguf")
        write_synthetic_gguf(p, "tiny-llama", ft, seed=0)
        out[ft] = p
    return out


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nats_llm_studio_amd.ops import _lib
    _lib.lib()   # fail loudly if the HIP library is missing on a GPU box
    return torch.device("cuda:0")
