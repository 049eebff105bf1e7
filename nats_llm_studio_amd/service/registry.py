"""Local model registry over the LM Studio on-disk tree `<MODELS_DIR>/<publisher>/<model>/*.gguf`.

Replaces LM Studio's `GET /api/v0/models` and `GET /api/v0/models/{id}` that the reference
calls (`/root/reference/nats_llm_studio.go:61-85`, `:136-156`). Entries are read from the
GGUF headers (architecture, file type, context length) and emitted in LM Studio REST v0
shape: {"object":"list","data":[{id, object, type, publisher, arch, compatibility_type,
quantization, state, max_context_length, path}]}.

Unlike the reference's delete path (`:99-133`: publisher prefix guessing, doubled
publisher, cwd-relative dir for an empty MODELS_DIR) the registry maps every id to the
exact file and directory it was scanned from.
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..gguf.reader import read_metadata


@dataclass
class ModelEntry:
    id: str
    publisher: str
    model_dir: str            # directory name under the publisher
    path: str                 # .gguf file
    dir: str                  # absolute model directory
    arch: str = "unknown"
    quantization: str = "unknown"
    max_context_length: int = 0
    size_bytes: int = 0
    aliases: List[str] = field(default_factory=list)

    def to_api(self, loaded: bool) -> dict:
        return {
            "id": self.id,
            "object": "model",
            "type": "llm",
            "publisher": self.publisher,
            "arch": self.arch,
            "compatibility_type": "gguf",
            "quantization": self.quantization,
            "state": "loaded" if loaded else "not-loaded",
            "max_context_length": self.max_context_length,
            "path": os.path.relpath(self.path, os.path.dirname(os.path.dirname(self.dir))),
            "size_bytes": self.size_bytes,
        }


def model_id_for(model_dir: str) -> str:
    mid = model_dir
    for suf in ("-GGUF", "-gguf", "_GGUF"):
        if mid.endswith(suf):
            mid = mid[: -len(suf)]
    return mid.lower()


class Registry:
    def __init__(self, models_dir: str):
        self.models_dir = os.path.abspath(os.path.expanduser(models_dir))
        self._lock = threading.Lock()
        self._entries: Dict[str, ModelEntry] = {}
        self._alias: Dict[str, str] = {}
        self._cache: Dict[str, tuple] = {}   # path -> (mtime, size, meta)
        self.generation = 0                  # bumped whenever a scan finds a different set of entries
        self._t_scan = -1e9                  # monotonic time of the last scan

    def scan(self) -> List[ModelEntry]:
        entries: Dict[str, ModelEntry] = {}
        alias: Dict[str, str] = {}
        root = self.models_dir
        if os.path.isdir(root):
            for pub in sorted(os.listdir(root)):
                pdir = os.path.join(root, pub)
                if not os.path.isdir(pdir) or pub.startswith("."):
                    continue
                for mdir in sorted(os.listdir(pdir)):
                    d = os.path.join(pdir, mdir)
                    if not os.path.isdir(d):
                        continue
                    ggufs = sorted(f for f in os.listdir(d) if f.endswith(".gguf") and not f.endswith(".part"))
                    for i, f in enumerate(ggufs):
                        path = os.path.join(d, f)
                        e = self._entry(pub, mdir, d, path, f, i, len(ggufs))
                        if e is None:
                            continue
                        entries[e.id] = e
                        for a in e.aliases:
                            alias.setdefault(a.lower(), e.id)
        for e in getattr(self, "_extra", {}).values():       # added entries survive re-scans
            entries.setdefault(e.id, e)
            for a in [e.id] + list(e.aliases):
                alias.setdefault(a.lower(), e.id)
        sig = lambda es: {k: (e.path, e.size_bytes, e.max_context_length) for k, e in es.items()}  # noqa: E731
        with self._lock:
            if sig(entries) != sig(self._entries):
                self.generation += 1
            self._entries = entries
            self._alias = alias
            self._t_scan = time.monotonic()
        return list(entries.values())

    def _entry(self, pub, mdir, d, path, fname, idx, n) -> Optional[ModelEntry]:
        try:
            st = os.stat(path)
        except OSError:
            return None
        hit = self._cache.get(path)
        if hit and hit[0] == st.st_mtime and hit[1] == st.st_size:
            md = hit[2]
        else:
            try:
                md = read_metadata(path)
            except Exception:
                return None
            md = {k: v for k, v in md.items() if not k.startswith("tokenizer.")}
            self._cache[path] = (st.st_mtime, st.st_size, md)
        arch = str(md.get("general.architecture", "unknown"))
        mid = model_id_for(mdir)
        if n > 1 and idx > 0:
            mid = f"{mid}:{os.path.splitext(fname)[0].lower()}"
        stem = os.path.splitext(fname)[0]
        e = ModelEntry(
            id=mid, publisher=pub, model_dir=mdir, path=path, dir=d, arch=arch,
            quantization=str(md.get("__file_type_name__", "unknown")),
            max_context_length=int(md.get(f"{arch}.context_length", 0) or 0), size_bytes=st.st_size,
            aliases=[mid, f"{pub}/{mdir}", f"{pub}/{mid}", mdir, stem, f"{pub}/{mdir}/{fname}", f"{pub}/{stem}"],
        )
        return e

    def add(self, e: ModelEntry):
        """Register an entry that does not live under models_dir (e.g. a preloaded model)."""
        with self._lock:
            self._entries[e.id] = e
            for a in [e.id] + list(e.aliases):
                self._alias.setdefault(a.lower(), e.id)
        self._extra = getattr(self, "_extra", {})
        self._extra[e.id] = e
        self.generation += 1

    def resolve(self, ident: str) -> Optional[ModelEntry]:
        with self._lock:
            key = self._alias.get(ident.lower())
            if key is None:
                key = self._alias.get(model_id_for(ident))
            return self._entries.get(key) if key else None

    def entries(self) -> List[ModelEntry]:
        with self._lock:
            return list(self._entries.values())

    # list_models re-reads the tree at most this often (pull / delete / sync re-scan at once): a model copied
    # into MODELS_DIR by hand is listed within a second, and a burst of list requests costs one directory walk
    RESCAN_S = 1.0

    def refresh(self, max_age: float = None):
        if time.monotonic() - self._t_scan > (self.RESCAN_S if max_age is None else max_age):
            self.scan()

    def list_api(self, loaded_ids=(), max_age: float = None) -> dict:
        self.refresh(max_age)
        loaded = set(loaded_ids)
        return {"object": "list", "data": [e.to_api(e.id in loaded) for e in self.entries()]}

    def safe_dir(self, d: str) -> bool:
        """True if `d` is strictly inside MODELS_DIR (no deleting the tree root or escaping it)."""
        root = os.path.realpath(self.models_dir)
        real = os.path.realpath(d)
        return real != root and os.path.commonpath([root, real]) == root
