"""Native CLI (`nls-nats`, csrc/tools/nls_nats.cpp) and sanitizer builds of the natscore core
(race detection -- the reference has none, `go test -race` was never possible)."""
import json
import os
import subprocess
import tempfile

import pytest

from nats_llm_studio_amd import build
from nats_llm_studio_amd.natsio import Client, EmbeddedServer
from nats_llm_studio_amd.service.config import WorkerConfig
from nats_llm_studio_amd.service.service import Service


@pytest.fixture(scope="module")
def cli_bin():
    return build.build_tool()


def _run(binary, *args, timeout=60):
    r = subprocess.run([binary, *args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_cli_req_bench_and_object_store(cli_bin, tmp_path):
    srv = EmbeddedServer().start()
    cfg = WorkerConfig(nats_url=srv.url, models_dir=str(tmp_path / "models"), backend="stub")
    os.makedirs(cfg.models_dir)
    svc = Service(cfg).start()
    try:
        out = json.loads(_run(cli_bin, "--server", srv.url, "req", "lmstudio.list_models", "{}"))
        assert out["ok"] is True and out["data"]["http_status"] == 200
        b = json.loads(_run(cli_bin, "--server", srv.url, "bench", "lmstudio.health", "{}", "--n", "50"))
        assert b["n"] == 50 and 0 < b["p50_ms"] <= b["p99_ms"]
        # the README's bucket workflow: obj add / put --name <publisher>/<model>/<file> / ls / get
        f = tmp_path / "m.gguf"
        f.write_bytes(os.urandom(300_000))
        _run(cli_bin, "--server", srv.url, "obj", "add", "llm-models")
        info = json.loads(_run(cli_bin, "--server", srv.url, "obj", "put", "llm-models", str(f), "--name",
                               "pub/model-GGUF/m.gguf", "--chunk", "65536"))
        assert info["size"] == 300_000 and info["digest"].startswith("SHA-256=")
        ls = json.loads(_run(cli_bin, "--server", srv.url, "obj", "ls", "llm-models"))
        assert [o["name"] for o in ls] == ["pub/model-GGUF/m.gguf"]
        dst = tmp_path / "back.gguf"
        _run(cli_bin, "--server", srv.url, "obj", "get", "llm-models", "pub/model-GGUF/m.gguf", "-O", str(dst))
        assert dst.read_bytes() == f.read_bytes()
        # pull_model over NATS materialises it into the model tree
        r = json.loads(_run(cli_bin, "--server", srv.url, "req", "lmstudio.pull_model",
                            '{"identifier": "pub/model"}'))
        assert r["ok"] is True and r["data"]["local_paths"][0].endswith("pub/model-GGUF/m.gguf")
    finally:
        svc.stop()
        svc.client.close()
        srv.stop()


def test_cli_standalone_server(cli_bin):
    p = subprocess.Popen([cli_bin, "server", "--port", "0"], stdout=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline()
        url = line.split()[4]
        assert url.startswith("nats://127.0.0.1:")
        c = Client().connect(url)
        sub = c.subscribe("x.>")
        c.publish("x.y", b"hi")
        m = sub.next_msg(5)
        assert bytes(m.data) == b"hi"
        c.close()
    finally:
        p.terminate()
        assert p.wait(10) == 0


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_natscore_under_sanitizers(san):
    """natscore_stress (queue-group responders, concurrent muxed requests on one connection,
    wildcard pub/sub, auto-unsubscribe, forced reconnect, object store) under TSAN / ASAN+UBSAN."""
    d = tempfile.mkdtemp(prefix="nls_san_")
    # LLVM's runtime (ROCm clang++): GCC 11's libtsan does not intercept pthread_cond_clockwait
    # (std::condition_variable::wait_for) and reports a false "double lock"
    cxx = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(cxx):
        pytest.skip("clang++ with sanitizer runtimes not found")
    exe = build.build_tool(f"natscore_stress_{san.split(',')[0]}", "natscore_stress.cpp",
                           extra=("-g", "-O1", f"-fsanitize={san}", "-fno-omit-frame-pointer"), out_dir=d, cxx=cxx)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ThreadSanitizer" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]


def test_kernel_bindings_match_the_built_library():
    """Every ctypes signature in ops/_lib.py names a symbol the in-tree _kernels.so exports (a binding left
    behind by a reverted kernel fails the first GPU call of every process, not any CPU test)."""
    import shutil
    from nats_llm_studio_amd.ops import _lib
    if not os.path.exists(_lib.LIB_PATH) or shutil.which("nm") is None:
        pytest.skip("no built _kernels.so / nm")
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    assert sorted(set(_lib._SIGS) - exported) == []
