"""Model store: JetStream Object-Store bucket -> local tree materialisation, and deletion.

* pull_model (`/root/reference/nats_llm_studio.go:46-59` ran `lms get <id>` against the
  internet): here `identifier` names objects in the bucket laid out as
  `<publisher>/<model>/<file>.gguf` (`README.md:278-282`); every matching object is
  streamed (SHA-256 verified, resumable .part, atomic rename) to
  `<MODELS_DIR>/<publisher>/<model>/<file>.gguf`.
* sync_model_from_bucket (`README.md:284-318`, design only in the reference):
  {bucket, object_name, publisher, model_dir} -> `<MODELS_DIR>/<publisher>/<model_dir>/model.gguf`.
* delete: exact directory from the registry, path-safety checked, then rmtree.
"""
from __future__ import annotations

import os
import shutil
import time
from typing import Callable, List, Optional

from ..natsio import Client, ObjectStore


class PullError(Exception):
    def __init__(self, msg: str, output: str = ""):
        super().__init__(msg)
        self.output = output


def _match(identifier: str, name: str) -> bool:
    ident = identifier.strip("/").lower()
    n = name.lower()
    if n == ident:
        return True
    if n.startswith(ident + "/"):
        return True
    # "publisher/model" may refer to "publisher/model-GGUF/<file>"
    parts = n.split("/")
    if len(parts) >= 2 and "/".join(parts[:2]).replace("-gguf", "") == ident.replace("-gguf", ""):
        return True
    return False


def _safe_rel(name: str) -> List[str]:
    parts = [p for p in name.split("/") if p not in ("", ".", "..")]
    if len(parts) < 3:
        if len(parts) == 2:
            return [parts[0], os.path.splitext(parts[1])[0], parts[1]]
        if len(parts) == 1:
            return ["local", os.path.splitext(parts[0])[0], parts[0]]
        raise ValueError(f"bad object name {name!r}")
    return parts[:2] + [parts[-1]]


class ModelStore:
    def __init__(self, client: Optional[Client], models_dir: str, bucket: str = "llm-models"):
        self.client = client
        self.models_dir = os.path.abspath(os.path.expanduser(models_dir))
        self.bucket = bucket

    def _os(self, bucket: Optional[str] = None, timeout: float = 30.0) -> ObjectStore:
        """Per-operation timeout 30 s, or what is left of the caller's deadline when that is shorter."""
        if self.client is None:
            raise PullError("no NATS connection for the object store")
        return ObjectStore(self.client, bucket or self.bucket, timeout=max(0.05, min(30.0, timeout)))

    def pull(self, identifier: str, progress: Callable[[int, int], None] = None,
             deadline: Optional[float] = None) -> dict:
        """deadline: time.monotonic() bound of the whole pull (the handler's 10-minute context,
        `nats_llm_studio.go:251`); an expired pull keeps its .part files and resumes on the next call."""
        out_lines = []
        t0 = time.time()

        def left(grace: float = 0.0) -> float:
            """Seconds left (0: no deadline); raises once the deadline is within `grace` (an operation timed
            out on the remaining budget handed to it just now)."""
            if deadline is None:
                return 0.0
            r = deadline - time.monotonic()
            if r <= grace:
                raise PullError(f"failed to pull '{identifier}': context deadline exceeded", "\n".join(out_lines))
            return r
        try:
            store = self._os(timeout=left() or 30.0)
            objs = store.list()
        except Exception as e:
            left(0.25)
            raise PullError(f"failed to list bucket '{self.bucket}': {e}", "")
        matches = [o for o in objs if _match(identifier, o["name"]) and o["name"].lower().endswith(".gguf")]
        if not matches:
            raise PullError(f"model '{identifier}' not found in bucket '{self.bucket}'",
                            f"no objects matching {identifier!r} in bucket {self.bucket!r}")
        paths = []
        total = 0
        for o in matches:
            pub, mdir, fname = _safe_rel(o["name"])
            d = os.path.join(self.models_dir, pub, mdir)
            os.makedirs(d, exist_ok=True)
            dest = os.path.join(d, fname)
            if os.path.exists(dest) and os.path.getsize(dest) == o.get("size", -1):
                out_lines.append(f"{o['name']}: already present at {dest}")
                paths.append(dest)
                continue
            try:
                budget = left()
                self._os(timeout=budget or 30.0).get_file(o["name"], dest, True, progress, budget)
            except PullError:
                raise
            except Exception as e:
                left(0.25)
                raise PullError(f"failed to download '{o['name']}': {e}", "\n".join(out_lines))
            total += int(o.get("size", 0))
            out_lines.append(f"{o['name']}: {o.get('size', 0)} bytes -> {dest} ({o.get('digest', '')} verified)")
            paths.append(dest)
        dt = time.time() - t0
        out_lines.append(f"pulled {len(paths)} file(s), {total} bytes in {dt:.2f}s"
                         + (f" ({total / dt / 1e9:.2f} GB/s)" if dt > 0 and total else ""))
        return {"output": "\n".join(out_lines), "paths": paths, "bytes": total, "seconds": dt}

    def sync(self, bucket: str, object_name: str, publisher: str, model_dir: str, filename: str = "model.gguf",
             deadline: Optional[float] = None) -> dict:
        for part in (publisher, model_dir, filename):
            if not part or "/" in part or part in (".", ".."):
                raise PullError(f"invalid path component {part!r}")
        d = os.path.join(self.models_dir, publisher, model_dir)
        os.makedirs(d, exist_ok=True)
        dest = os.path.join(d, filename)
        t0 = time.time()
        budget = 0.0
        if deadline is not None:
            budget = deadline - time.monotonic()
            if budget <= 0:
                raise PullError("context deadline exceeded")
        info = self._os(bucket, budget or 30.0).get_file(object_name, dest, True, None, budget)
        return {"local_path": dest, "size": info.get("size"), "digest": info.get("digest"),
                "seconds": time.time() - t0}

    def push(self, path: str, object_name: str, bucket: Optional[str] = None, chunk_size: int = 128 * 1024) -> dict:
        store = self._os(bucket)
        try:
            store.create("LLM model repository (.gguf)")
        except Exception:
            pass
        return store.put_file(object_name, path, chunk_size)

    @staticmethod
    def remove_dir(d: str):
        shutil.rmtree(d)
