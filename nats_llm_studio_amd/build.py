"""Build the native parts in-tree (no JIT cache, no site-packages):

* `_kernels.so`  -- gfx950 HIP kernels (hipcc --offload-arch=gfx950)
* `_natscore.*.so` -- C++ NATS wire core (client + embedded server + JetStream object store), pybind11

    python -m nats_llm_studio_amd.build [--force]
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def source_hash(srcs, flags=()) -> str:
    """sha256 over the sources' names + contents and the compile flags: what a built library is
    stamped with (`<lib>.srchash`), so staleness is decided by content, not by file times (a fresh
    checkout or a copied tree has arbitrary mtimes)."""
    h = hashlib.sha256()
    for f in sorted(srcs):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _stamp(out: str) -> str:
    return out + ".srchash"


def read_stamp(out: str):
    try:
        with open(_stamp(out)) as f:
            return json.load(f).get("hash")
    except (OSError, ValueError):
        return None


def _stale(out: str, srcs, flags=()) -> bool:
    return not os.path.exists(out) or read_stamp(out) != source_hash(srcs, flags)


def _write_stamp(out: str, srcs, flags=()):
    with open(_stamp(out), "w") as f:
        json.dump({"hash": source_hash(srcs, flags), "files": sorted(os.path.basename(s) for s in srcs)}, f)


def kernel_sources():
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    return srcs, srcs + sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))


def kernel_flags(defines=()):
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", *[f"-D{d}" for d in defines]]


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build_kernels(force: bool = False, defines=(), tag: str = "") -> str:
    """Compile each .hip translation unit to an object in parallel, then link one .so.
    `defines` + `tag`: an A/B variant library `_kernels_<tag>.so` (e.g. tools/gemm_ab.py), built in
    its own object directory; the default build is `_kernels.so`."""
    out = os.path.join(PKG, f"_kernels_{tag}.so" if tag else "_kernels.so")
    srcs, deps = kernel_sources()
    flags = kernel_flags(defines)
    if force or _stale(out, deps, flags):
        from concurrent.futures import ThreadPoolExecutor
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        bdir = os.path.join(ROOT, "build", f"kernels_{tag}" if tag else "kernels")
        os.makedirs(bdir, exist_ok=True)
        hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
        objs = [os.path.join(bdir, os.path.basename(s) + ".o") for s in srcs]
        jobs = [(s, o) for s, o in zip(srcs, objs) if force or _stale(o, [s] + hdrs, flags)]

        def compile_one(so):
            _run([hipcc, *flags, "-c", so[0], "-o", so[1]])
            _write_stamp(so[1], [so[0]] + hdrs, flags)

        with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
            list(ex.map(compile_one, jobs))
        tmp = out + ".tmp"
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", *objs, "-o", tmp])
        os.replace(tmp, out)
        _write_stamp(out, deps, flags)
    return out


def kernels_current(out: str = None) -> bool:
    """True when the in-tree `_kernels.so` was built from exactly the current kernel sources."""
    out = out or os.path.join(PKG, "_kernels.so")
    srcs, deps = kernel_sources()
    return os.path.exists(out) and read_stamp(out) == source_hash(deps, kernel_flags())


def natscore_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "natsio", "_natscore" + suffix)


def build_natscore(force: bool = False) -> str:
    out = natscore_path()
    srcs = sorted(glob.glob(os.path.join(CSRC, "natscore", "*.cpp")))
    if not srcs:
        return ""
    deps = srcs + glob.glob(os.path.join(CSRC, "natscore", "*.h"))
    if force or _stale(out, deps):
        import pybind11
        inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{os.path.join(CSRC, 'natscore')}"]
        tmp = out + ".tmp"
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-fvisibility=hidden", *inc, *srcs,
              "-o", tmp, "-lssl", "-lcrypto"])      # libssl: NATS TLS; libcrypto: ed25519 nkey signatures
        os.replace(tmp, out)
        _write_stamp(out, deps)
    return out


def tokcore_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "tokenizer", "_tokcore" + suffix)


def build_tokcore(force: bool = False) -> str:
    """The native BPE merge loops of the tokenizers (csrc/tokcore), pybind11."""
    out = tokcore_path()
    srcs = sorted(glob.glob(os.path.join(CSRC, "tokcore", "*.cpp")))
    if not srcs:
        return ""
    if force or _stale(out, srcs):
        import pybind11
        inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
        tmp = out + ".tmp"
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", *inc, *srcs, "-o", tmp])
        os.replace(tmp, out)
        _write_stamp(out, srcs)
    return out


def _natscore_lib_srcs():
    return [s for s in sorted(glob.glob(os.path.join(CSRC, "natscore", "*.cpp"))) if not s.endswith("bindings.cpp")]


def build_tool(name: str = "nls-nats", src: str = "nls_nats.cpp", extra=(), out_dir: str = None,
               force: bool = False, cxx: str = "g++") -> str:
    """Native executables over natscore (no Python): the `nls-nats` CLI (server / req / obj ...)."""
    out = os.path.join(out_dir or os.path.join(ROOT, "bin"), name)
    srcs = [os.path.join(CSRC, "tools", src)] + _natscore_lib_srcs()
    deps = srcs + glob.glob(os.path.join(CSRC, "natscore", "*.h"))
    if force or _stale(out, deps):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        tmp = out + ".tmp"
        _run([cxx, "-O2", "-std=c++17", "-pthread", f"-I{os.path.join(CSRC, 'natscore')}", *extra, *srcs,
              "-o", tmp, "-lssl", "-lcrypto"])
        os.replace(tmp, out)
        _write_stamp(out, deps)
    return out


def build_diag(force: bool = False):
    """Stand-alone gfx950 probe libraries of tools/diag (csrc/diag/<name>.hip -> tools/diag/_<name>.so)."""
    outs = []
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    for src in sorted(glob.glob(os.path.join(CSRC, "diag", "*.hip"))):
        out = os.path.join(ROOT, "tools", "diag", "_" + os.path.basename(src)[:-4] + ".so")
        flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared"]
        if force or _stale(out, [src], flags):
            tmp = out + ".tmp"
            _run([hipcc, *flags, src, "-o", tmp])
            os.replace(tmp, out)
            _write_stamp(out, [src], flags)
        outs.append(out)
    return outs


def build_all(force: bool = False):
    k = build_kernels(force)
    n = build_natscore(force)
    build_tokcore(force)
    build_tool(force=force)
    build_diag(force)
    return k, n


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
