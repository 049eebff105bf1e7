"""Chat backends behind `lmstudio.chat_model`.

* `EngineBackend` -- the co-located GPU engine (JIT load on first chat like LM Studio,
  LRU unload, continuous batching across concurrent requests).
* `StubBackend`  -- CPU echo backend (BASELINE config 1: "embedded nats-server with CPU stub
  backend (granite-3.0-2b echo), no GPU"), same response shape, no model weights.

Both produce LM Studio `/api/v0/chat/completions` bodies (what the reference embeds raw
under data.response, `/root/reference/nats_llm_studio.go:356-363`).
"""
from __future__ import annotations

import collections
import os
import threading
import time
import uuid
from typing import Callable, Dict, Optional

from .. import __version__
from .registry import ModelEntry

Done = Callable[..., None]      # (http_status, body[, trace marks])


def _error_body(msg: str) -> dict:
    return {"error": msg}


def chat_response(model_id: str, entry: Optional[ModelEntry], text: str, prompt_tokens: int,
                  completion_tokens: int, finish_reason: str, stop_reason: str, ttft: float, gen_time: float,
                  ctx: int, arch: str = "", quant: str = "") -> dict:
    tps = completion_tokens / gen_time if gen_time > 0 else 0.0
    return {
        "id": f"chatcmpl-{uuid.uuid4().hex[:24]}",
        "object": "chat.completion",
        "created": int(time.time()),
        "model": model_id,
        "choices": [{"index": 0, "logprobs": None, "finish_reason": finish_reason,
                     "message": {"role": "assistant", "content": text}}],
        "usage": {"prompt_tokens": prompt_tokens, "completion_tokens": completion_tokens,
                  "total_tokens": prompt_tokens + completion_tokens},
        "stats": {"tokens_per_second": round(tps, 3), "time_to_first_token": round(ttft, 6),
                  "generation_time": round(gen_time, 6), "stop_reason": stop_reason},
        "model_info": {"arch": arch or (entry.arch if entry else ""),
                       "quant": quant or (entry.quantization if entry else ""),
                       "format": "gguf", "context_length": ctx},
        "runtime": {"name": "nats-llm-studio-amd", "version": __version__, "supported_formats": ["gguf"]},
    }


def _messages(req: dict):
    msgs = req.get("messages")
    if not isinstance(msgs, list) or not msgs:
        raise ValueError("'messages' must be a non-empty array")
    for m in msgs:
        if not isinstance(m, dict) or "role" not in m:
            raise ValueError("each message needs a 'role'")
    return msgs



class DeadlineExceeded(Exception):
    """A handler's context expired (Go: context.DeadlineExceeded, "context deadline exceeded")."""

class StubBackend:
    """Echo backend: returns the last user message (token counts = whitespace words)."""

    name = "stub"

    def __init__(self, default_model: str = "granite-3.0-2b-instruct"):
        self.default_model = default_model
        self.requests = 0

    def loaded_ids(self):
        return [self.default_model]

    def chat(self, model_id: str, entry: Optional[ModelEntry], req: dict, done: Done, deadline: float = None,
             stream_cb=None):
        self.requests += 1
        try:
            msgs = _messages(req)
        except ValueError as e:
            done(400, _error_body(str(e)))
            return
        t0 = time.perf_counter()
        last = next((m.get("content", "") for m in reversed(msgs) if m.get("role") == "user"), "")
        if isinstance(last, list):
            last = "".join(p.get("text", "") for p in last if isinstance(p, dict))
        prompt_tokens = sum(len(str(m.get("content", "")).split()) for m in msgs)
        mt = req.get("max_tokens")
        words = str(last).split()
        if isinstance(mt, int) and mt >= 0:
            words = words[:mt]
        text = " ".join(words)
        if stream_cb:
            stream_cb(text)
        dt = time.perf_counter() - t0
        done(200, chat_response(model_id, entry, text, prompt_tokens, len(words), "stop", "eosFound", dt, dt, 4096,
                                arch="granite", quant="stub"))

    def unload(self, model_id: str) -> bool:
        return False

    def stats(self):
        return {"backend": "stub", "requests": self.requests}


class EngineBackend:
    """GGUF models served by the HIP engine; JIT-loaded, LRU-evicted.

    Loading never holds the registry lock: a model is built outside it (concurrent chats for the
    same model wait on one per-model future), so `list_models` / `health` / chats of loaded models
    keep answering during a tens-of-seconds load. Loads of DIFFERENT models are serialised by a
    separate build mutex, and each evicts before it builds: two first requests for two models never
    size their weights / KV pools against each other's half-finished allocations, and a model being
    built counts toward `max_loaded_models`. Every chat pins its model state (`inflight`); an evicted
    or deleted model is unloaded only when its last in-flight chat has finished."""

    name = "engine"

    def __init__(self, cfg):
        self.cfg = cfg
        self._lock = threading.RLock()
        self._build_lock = threading.Lock()   # one model build at a time (device memory is sized at build)
        self._loaded: "collections.OrderedDict[str, dict]" = collections.OrderedDict()
        self._loading: Dict[str, list] = {}    # model id -> [build Future, chats waiting on it]
        self._ids: tuple = ()          # lock-free snapshot of the loaded model ids
        self._device = None
        self.pinned = False          # tensor-parallel worker: serves only its preloaded model

    def device(self):
        import torch
        if self._device is None:
            d = self.cfg.device
            if d == "auto":
                d = "cuda:0" if torch.cuda.is_available() else "cpu"
            self._device = torch.device(d)
        return self._device

    def loaded_ids(self):
        return list(self._ids)

    def _publish(self):
        self._ids = tuple(self._loaded)

    def build_state(self, entry: ModelEntry, shard=None, comm=None, start: bool = True) -> dict:
        """GGUF -> device model + tokenizer + chat template + engine (one TP shard if `shard`)."""
        from ..engine.engine import Engine
        from ..gguf.reader import GGUFReader
        from ..models.llama import LlamaModel, ShardSpec
        from ..tokenizer.bpe import tokenizer_from_metadata
        from ..tokenizer.chat_template import ChatTemplate, default_template
        t0 = time.time()
        reader = GGUFReader(entry.path)
        md = reader.metadata
        model = LlamaModel(reader, self.device(), shard or ShardSpec(), comm)
        tok = tokenizer_from_metadata(md)
        tmpl = md.get("tokenizer.chat_template") or default_template(model.cfg.arch,
                                                                     md.get("tokenizer.ggml.model", "gpt2"))
        bos = tok.tokens[tok.bos_id] if tok.bos_id is not None else ""
        eos = tok.tokens[tok.eos_id] if tok.eos_id is not None else ""
        # EP: prefill chunks stay within the IPC row exchange's token budget (larger ones take the all-to-all)
        mp = min(self.cfg.max_prefill_tokens, 2048) if model.ep else self.cfg.max_prefill_tokens
        eng = Engine(model, tok, max_batch=self.cfg.max_batch, ctx=self.cfg.max_ctx or None,
                     kv_mem_fraction=self.cfg.kv_mem_fraction, max_prefill_tokens=mp)
        if eng.use_graphs and os.environ.get("NLS_CAPTURE_AT_LOAD", "1") == "1":
            eng.capture_all()      # every decode bucket's graphs now, not inside the first request burst
        if start:
            eng.start()
        return {"engine": eng, "tok": tok, "tmpl": ChatTemplate(tmpl, bos, eos), "entry": entry,
                "load_s": time.time() - t0, "inflight": 0, "evicted": False}

    def adopt(self, st: dict, pinned: bool = True):
        """Serve an already-built state (tensor-parallel rank 0); other models are refused."""
        st.setdefault("inflight", 0)
        st.setdefault("evicted", False)
        with self._lock:
            self._loaded[st["entry"].id] = st
            self.pinned = pinned
            self._publish()

    def _evict_locked(self, keep: int) -> list:
        """Drop LRU models until at most `keep` remain; returns the idle ones to unload now."""
        idle = []
        while len(self._loaded) > keep:
            _, st = self._loaded.popitem(last=False)
            st["evicted"] = True
            if st["inflight"] == 0:
                idle.append(st)
        self._publish()
        return idle

    def load(self, entry: ModelEntry) -> dict:
        """The model's state, pinned for one chat (pair with `release`)."""
        from concurrent.futures import Future
        while True:
            with self._lock:
                st = self._loaded.get(entry.id)
                if st is not None:
                    self._loaded.move_to_end(entry.id)
                    st["inflight"] += 1
                    return st
                if self.pinned:
                    raise RuntimeError(f"this tensor-parallel worker serves only {list(self._loaded)}")
                slot = self._loading.get(entry.id)
                owner = slot is None
                if owner:
                    slot = self._loading[entry.id] = [Future(), 0]
                else:
                    slot[1] += 1        # the owner pins the state for this waiter when the build lands
                fut = slot[0]
            if not owner:
                # another chat is loading this model: the state arrives already pinned for this chat, so a
                # build of another model that evicts right after this one cannot take it away in between
                return fut.result()
            try:
                with self._build_lock:
                    with self._lock:    # evict under the build mutex: the slot this build takes is free
                        idle = self._evict_locked(max(1, self.cfg.max_loaded_models) - 1)
                    for old in idle:
                        old["engine"].unload()
                    st = self.build_state(entry)
            except BaseException as e:
                with self._lock:
                    self._loading.pop(entry.id, None)
                fut.set_exception(e)
                raise
            with self._lock:
                idle = self._evict_locked(max(1, self.cfg.max_loaded_models) - 1)
                self._loaded[entry.id] = st
                st["inflight"] += 1 + slot[1]       # this chat and every chat waiting on the build
                self._publish()
                self._loading.pop(entry.id, None)
            for old in idle:
                old["engine"].unload()
            fut.set_result(st)
            return st

    def _load_until(self, entry: ModelEntry, deadline: Optional[float]) -> dict:
        """load(), bounded by the request's monotonic deadline: a cold build runs on a helper thread and the
        caller gives up (DeadlineExceeded) when the deadline passes first; a build that completes after that
        releases the pin it took for the abandoned request."""
        if deadline is None or entry.id in self._ids:
            return self.load(entry)
        lk, ev, box = threading.Lock(), threading.Event(), {}

        def run():
            try:
                st, err = self.load(entry), None
            except BaseException as e:          # noqa: BLE001 -- handed to the waiting request
                st, err = None, e
            with lk:
                if box.get("abandoned"):
                    if st is not None:
                        self.release(st)
                    return
                box.update(st=st, err=err)
                ev.set()
        threading.Thread(target=run, name=f"nls-load-{entry.id}", daemon=True).start()
        ev.wait(max(0.0, deadline - time.monotonic()))
        with lk:
            if not ev.is_set():
                box["abandoned"] = True
                raise DeadlineExceeded(entry.id)
        if box["err"] is not None:
            raise box["err"]
        return box["st"]

    def release(self, st: dict):
        with self._lock:
            st["inflight"] -= 1
            gone = st["evicted"] and st["inflight"] == 0
        if gone:
            st["engine"].unload()

    def unload(self, model_id: str) -> bool:
        with self._lock:
            if self.pinned:
                return False
            st = self._loaded.pop(model_id, None)
            self._publish()
            if st is None:
                return False
            st["evicted"] = True
            idle = st["inflight"] == 0
        if idle:
            st["engine"].unload()
        return True

    def chat(self, model_id: str, entry: Optional[ModelEntry], req: dict, done: Done, deadline: float = None,
             stream_cb=None):
        from ..engine.engine import GenRequest
        from ..engine.sampling import SamplingParams
        if entry is None:
            done(404, _error_body(f"Model '{model_id}' not found"))
            return
        try:
            msgs = _messages(req)
        except ValueError as e:
            done(400, _error_body(str(e)))
            return
        try:
            st = self._load_until(entry, deadline)
        except DeadlineExceeded:
            # the chat's context (reference: 2 min from receipt, `nats_llm_studio.go:328`) expired during a
            # cold JIT load: reply now; the build goes on and serves the next request
            done(0, _error_body("context deadline exceeded"))
            return
        except Exception as e:
            done(500, _error_body(f"failed to load model '{model_id}': {e}"))
            return
        released = [False]

        def release():
            if not released[0]:
                released[0] = True
                self.release(st)

        try:
            eng, tok, tmpl = st["engine"], st["tok"], st["tmpl"]
            try:
                prompt = tmpl.render(msgs, add_generation_prompt=True)
            except Exception as e:
                release()
                done(400, _error_body(f"chat template error: {e}"))
                return
            ids = tok.encode(prompt, add_bos=False)
            params = SamplingParams.from_request(req, default_max=self.cfg.default_max_tokens)
            on_token = None
            if stream_cb is not None:
                from ..tokenizer.bpe import StreamDecoder
                sd = StreamDecoder(tok)

                def on_token(t, _sd=sd):
                    d = _sd.push(t)
                    if d:
                        stream_cb(d)
            fut = eng.submit(GenRequest(ids, params, on_token=on_token, deadline=deadline))
            ctx = eng.ctx
        except Exception as e:
            release()
            done(500, _error_body(f"generation failed: {e}"))
            return

        def finished(f):
            release()
            try:
                r = f.result()
            except Exception as e:
                done(400, _error_body(str(e)))
                return
            if r.finish_reason == "error":
                done(500, _error_body(r.error or "generation failed"))
                return
            if r.finish_reason == "cancelled":     # engine stopped under the request (unload / shutdown)
                done(503, _error_body(f"generation cancelled: model '{model_id}' was unloaded"))
                return
            if r.finish_reason == "timeout":       # handler context expired (reference: 2 min, `:328`)
                done(0, _error_body("context deadline exceeded"))
                return
            done(200, chat_response(model_id, entry, r.text, r.prompt_tokens, r.completion_tokens,
                                    "length" if r.finish_reason == "length" else "stop", r.stop_reason,
                                    r.time_to_first_token, r.generation_time, ctx),
                 {"queued": r.t_submit, "admitted": r.t_admit, "first_token": r.t_first, "done": r.t_done,
                  "request_id": r.request_id})
        fut.add_done_callback(finished)

    def stats(self):
        with self._lock:
            items = list(self._loaded.items())
        return {"backend": "engine", "device": str(self._device),
                "loading": list(self._loading),
                "models": {k: dict(v["engine"].stats(), load_s=round(v["load_s"], 3), inflight=v["inflight"])
                           for k, v in items}}


class HttpBackend:
    """The reference's own mode: forward to an LM Studio server (`LMSTUDIO_BASE_URL`).

    ListModels / Chat semantics of `/root/reference/nats_llm_studio.go:136-179`: the raw
    body and the HTTP status are returned WITHOUT checking the status (a non-200 still
    yields ok:true with http_status); the chat payload is forwarded verbatim with
    Content-Type application/json; a 2-minute client timeout (`:36`)."""

    name = "http"

    def __init__(self, base_url: str, timeout: float = 120.0):
        self.base = base_url.rstrip("/")
        self.timeout = timeout
        self.requests = 0

    def _do(self, method: str, path: str, body: Optional[bytes] = None, timeout: Optional[float] = None):
        """One HTTP exchange under a TOTAL deadline (the reference's context / http.Client timeout bound the whole
        request, `nats_llm_studio.go:36`, `:229`): urllib's `timeout` is per socket operation, so a slow-dripping
        server could run past it. The exchange runs on a daemon thread and the caller waits at most `t`; the
        thread itself re-arms the socket timeout to what is left before every read, so it ends soon after."""
        import urllib.error
        import urllib.request
        req = urllib.request.Request(self.base + path, data=body, method=method)
        if body is not None:
            req.add_header("Content-Type", "application/json")
        t = self.timeout if timeout is None else min(self.timeout, timeout)
        deadline = time.monotonic() + t
        box = {}

        def read_all(r):
            sock = getattr(getattr(getattr(r, "fp", None), "raw", None), "_sock", None)
            parts = []
            while True:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError("context deadline exceeded")
                if sock is not None:
                    try:
                        sock.settimeout(left)
                    except OSError:
                        pass
                b = r.read(1 << 16)
                if not b:
                    return b"".join(parts)
                parts.append(b)

        def run():
            try:
                with urllib.request.urlopen(req, timeout=t) as r:
                    box["v"] = (r.status, read_all(r))
            except urllib.error.HTTPError as e:       # non-2xx: body + status, not an error
                try:
                    box["v"] = (e.code, read_all(e))
                except BaseException as e2:
                    box["e"] = e2
            except BaseException as e:
                box["e"] = e
        th = threading.Thread(target=run, name="nls-http", daemon=True)
        th.start()
        th.join(max(0.0, deadline - time.monotonic()))
        if th.is_alive() or not box:
            raise TimeoutError("context deadline exceeded")
        if "e" in box:
            raise box["e"]
        return box["v"]

    def list_models_raw(self, timeout: Optional[float] = None):
        return self._do("GET", "/api/v0/models", timeout=timeout)

    def chat_raw(self, payload: bytes):
        self.requests += 1
        return self._do("POST", "/api/v0/chat/completions", payload)

    def loaded_ids(self):
        return []

    def unload(self, model_id: str) -> bool:
        return False

    def stats(self):
        return {"backend": "http", "base_url": self.base, "requests": self.requests}
