"""The NATS service: the reference's four subjects (+ the README's bucket sync, metrics, health).

Subjects (prefix `lmstudio`, `README.md:17-21`), each joined with queue group
NATS_QUEUE_GROUP (`README.md:475-484` -- documented but never coded in the reference,
whose `Server` never subscribes, `nats_llm_studio.go:181-205`):

  lmstudio.list_models            -> onListModels   (`nats_llm_studio.go:228-248`)
  lmstudio.pull_model             -> OnPullModel    (`:250-286`)
  lmstudio.delete_model           -> OnDeleteModel  (`:288-324`)
  lmstudio.chat_model             -> OnChatModel    (`:327-364`)
  lmstudio.sync_model_from_bucket -> README.md:284-318 (design only in the reference)
  lmstudio.metrics / lmstudio.health (observability; new)

Validation order, error strings and envelope shapes are the reference's. Chat requests
do not block a handler thread: they are handed to the continuous-batching engine and the
reply is published from the completion callback, so one worker serves many concurrent chats
(the reference serialises one generation per subscription).
"""
from __future__ import annotations

import json
import os
import threading
import time
from collections import defaultdict
from typing import Optional

from . import envelope
from .backends import EngineBackend, HttpBackend, StubBackend
from .config import WorkerConfig
from .registry import Registry
from .store import ModelStore, PullError
from ..natsio import Client
from ..utils.metrics import LatencyHistogram
from ..utils.tracing import Tracer


def _is_timeout(e: BaseException) -> bool:
    import socket
    return isinstance(e, (socket.timeout, TimeoutError)) or isinstance(getattr(e, "reason", None),
                                                                         (socket.timeout, TimeoutError))


class Service:
    def __init__(self, cfg: WorkerConfig, client: Optional[Client] = None, backend=None):
        self.cfg = cfg
        self.client = client
        self.registry = Registry(cfg.models_dir)
        if backend is None:
            if cfg.backend == "stub":
                backend = StubBackend()
            elif cfg.backend == "http":
                backend = HttpBackend(cfg.lmstudio_base_url, cfg.timeout_chat)
            else:
                backend = EngineBackend(cfg)
        self.backend = backend
        self.store: Optional[ModelStore] = None
        self.subs = []
        self.t_start = time.time()
        self.counters = defaultdict(int)
        self.latency = defaultdict(LatencyHistogram)
        self.tracer = Tracer()
        self._lock = threading.Lock()
        self._unloads = {}            # model id -> daemon thread of the delete handler's bounded unload
        self._list_cache = {}         # (registry generation, loaded ids) -> encoded list_models reply
        self._list_sub = None         # the list_models subscription while its replies are native (auto-reply)
        self._list_key = None         # cache key of the body the native responder holds
        self._list_stop = threading.Event()
        self._list_thread = None
        self._list_lock = threading.Lock()   # orders body updates against native_list(False)

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "Service":
        if self.client is None:
            self.client = Client().connect(self.cfg.nats_url, name=f"nats-llm-studio-amd-{os.getpid()}",
                                           **self.cfg.nats_auth())
        self.store = ModelStore(self.client, self.cfg.models_dir, self.cfg.bucket)
        self.registry.scan()
        q = self.cfg.queue_group
        w = self.cfg.handler_workers
        routes = [
            ("list_models", self.on_list_models, w),
            ("pull_model", self.on_pull_model, 2),
            ("delete_model", self.on_delete_model, 2),
            ("chat_model", self.on_chat_model, w),
            ("sync_model_from_bucket", self.on_sync_model_from_bucket, 2),
            ("metrics", self.on_metrics, 1),
            ("health", self.on_health, 1),
        ]
        for name, fn, workers in routes:
            self.subs.append(self.client.subscribe(self.cfg.subject(name), q, self._wrap(name, fn), workers))
            if name == "list_models" and self.cfg.native_list_models and not isinstance(self.backend, HttpBackend):
                self._list_sub = self.subs[-1]
        if self._list_sub is not None:
            # the registry listing is a cached read: the client's reader thread answers it (no Python on the RTT
            # path), the body rebuilt before a reply whose request changed the registry or the loaded set (a pull /
            # delete / JIT-loading chat reply is followed by a listing that shows it; see respond()) and every
            # list_refresh_ms on the refresher thread (rescans of MODELS_DIR, loads, unloads)
            self._publish_list_reply()
            self._list_stop.clear()
            self._list_thread = threading.Thread(target=self._list_refresher, name="nls-list-reply", daemon=True)
            self._list_thread.start()
        self.client.flush()
        return self

    def native_list(self, enabled: bool):
        """Switch list_models between the native responder and the Python handler at run time (the handler keeps
        the reference's 30 s read deadline; the native reply is the last snapshot, refreshed every list_refresh_ms)."""
        sub = next((x for x in self.subs if x.subject == self.cfg.subject("list_models")), None)
        if sub is None or isinstance(self.backend, HttpBackend):
            return
        if enabled:
            with self._list_lock:
                self._list_sub, self._list_key = sub, None
            self._publish_list_reply()
        else:
            with self._list_lock:
                self._list_sub = None
                sub.set_auto_reply(None)

    def _list_body(self, rescan: bool = True):
        """(cache key, encoded list_models reply) of the current registry snapshot and loaded set. `rescan`
        lets the registry re-walk MODELS_DIR when its last scan is stale; reply paths pass False."""
        loaded = tuple(self.backend.loaded_ids())
        if rescan:
            self.registry.refresh()
        key = (self.registry.generation, loaded)
        body = self._list_cache.get(key)
        if body is None:
            # the encoded reply of an unchanged snapshot is reused (one per registry generation + loaded set)
            body = envelope.ok({"http_status": 200, "models": self.registry.list_api(loaded)})
            self._list_cache = {key: body}
        return key, body

    def _publish_list_reply(self, rescan: bool = True):
        """Install the current listing in the native responder. The snapshot is built and stored under ONE
        lock, so a refresher snapshot taken before a pull / delete can never overwrite the newer one a reply
        path installed after it (the last writer always holds the newest registry state)."""
        if self._list_sub is None:
            return
        with self._list_lock:
            sub = self._list_sub
            if sub is None:
                return
            try:
                key, body = self._list_body(rescan)
            except Exception:
                key, body = None, None      # a registry read that fails goes back to the handler (its error reply)
            if key is not None and key == self._list_key:
                return
            try:
                sub.set_auto_reply(body)
                self._list_key = key
            except Exception:
                self._list_key = None

    def _listing_stale(self) -> bool:
        """Cheap check on the reply path: did the loaded set or the registry generation move since the
        installed body was built? (No directory walk: rescans belong to the refresher thread.)"""
        k = self._list_key
        if k is None:
            return True
        try:
            return k[0] != self.registry.generation or k[1] != tuple(self.backend.loaded_ids())
        except Exception:
            return True

    def _list_refresher(self):
        period = max(0.005, self.cfg.list_refresh_ms / 1e3)
        while not self._list_stop.wait(period):
            self._publish_list_reply()

    def stop(self):
        self._list_stop.set()
        if self._list_thread is not None:
            self._list_thread.join(timeout=2)
            self._list_thread = None
        self._list_sub = None
        for s in self.subs:
            s.unsubscribe()
        self.subs.clear()
        if hasattr(self.backend, "loaded_ids"):
            for mid in list(self.backend.loaded_ids()):
                try:
                    self.backend.unload(mid)
                except Exception:
                    pass

    def _wrap(self, name, fn):
        def handler(msg):
            t0 = time.perf_counter()
            with self._lock:
                self.counters[name] += 1
            try:
                fn(msg)
            finally:
                self.latency[name].add(time.perf_counter() - t0)
        return handler

    def _unload_bounded(self, model_id: str, deadline: Optional[float]) -> bool:
        """The engine unload under the delete handler's context, like `lms unload` under
        exec.CommandContext (`nats_llm_studio.go:87-97`): it runs on the service's one persistent unload
        thread (no thread per request) and a call still running at the deadline is logged and left to
        finish -- the unload is best effort in the reference too. True when it finished in time.

        Each call gets its own daemon thread (like each `lms unload` being its own process): an unload that
        hangs never queues later deletes behind it and never blocks interpreter exit. While a previous unload
        of the SAME model is still running, no second one is started (it would only wait on the first)."""
        if deadline is None:
            self.backend.unload(model_id)
            return True
        with self._lock:
            prev = self._unloads.get(model_id)
            if prev is None or not prev.is_alive():
                box = {}

                def run(_m=model_id, _b=box):
                    try:
                        self.backend.unload(_m)
                    except BaseException as e:
                        _b["e"] = e
                prev = threading.Thread(target=run, name="nls-unload", daemon=True)
                prev.box = box
                self._unloads[model_id] = prev
                prev.start()
        prev.join(max(0.0, deadline - time.monotonic()))
        err = "context deadline exceeded" if prev.is_alive() else prev.box.get("e")
        if err is not None:                       # timeout, or the unload itself failed: logged, not fatal
            print(f"warning: failed to unload model {model_id}: {err}", flush=True)
            return False
        return True

    def respond(self, msg, body: bytes, changed: bool = False):
        """respondJSON (`nats_llm_studio.go:207-217`): log (not raise) when there is no reply subject.

        A listing requested after this reply sees what this request changed: handlers that change the
        registry (pull, delete, sync) pass `changed` and the native listing is rebuilt before the reply goes
        out; any other reply only compares the installed body's key with the registry generation and the
        loaded set (a chat's JIT load) -- no directory walk on the chat reply path."""
        if not msg.reply:
            print(f"error responding to NATS message: nats: message does not have a reply", flush=True)
            return
        if self._list_sub is not None and (changed or self._listing_stale()):
            self._publish_list_reply(rescan=False)
        try:
            self.client.publish(msg.reply, body)
        except Exception as e:
            print(f"error responding to NATS message: {e}", flush=True)

    # ------------------------------------------------------------------ handlers
    def _raw_json(self, body: bytes):
        """json.RawMessage: a non-JSON backend body makes marshalling fail -> literal fallback."""
        try:
            return json.loads(body.decode("utf-8") if body else "")
        except (UnicodeDecodeError, ValueError):
            return None

    def on_list_models(self, msg):
        if isinstance(self.backend, HttpBackend):           # `nats_llm_studio.go:228-248`
            try:
                # the 30 s context bounds the HTTP call itself (no helper thread)
                status, body = self.backend.list_models_raw(timeout=self.cfg.timeout_list or None)
            except Exception as e:
                if _is_timeout(e):
                    e = "context deadline exceeded"
                self.respond(msg, envelope.error(f"error calling LM Studio: {e}", {"http_status": 0}))
                return
            raw = self._raw_json(body)
            self.respond(msg, envelope.FALLBACK if raw is None else
                         envelope.ok({"http_status": status, "models": raw}))
            return
        # an in-memory registry snapshot: read inline on the handler thread (the RTT path of BASELINE config 1)
        # and held to the 30 s context afterwards -- a thread per request cost ~0.1 ms of the ~0.08 ms RTT
        t0 = time.monotonic()
        try:
            _, body = self._list_body()
        except Exception as e:
            self.respond(msg, envelope.error(f"error reading model registry: {e}", {"http_status": 0}))
            return
        if self.cfg.timeout_list and time.monotonic() - t0 > self.cfg.timeout_list:
            self.respond(msg, envelope.error("error reading model registry: context deadline exceeded",
                                             {"http_status": 0}))
            return
        self.respond(msg, body)

    def on_pull_model(self, msg):
        err = envelope.go_json_error(msg.data, "PullModelRequest", {"identifier": "Identifier"})
        if err:
            self.respond(msg, envelope.error(f"invalid JSON in PullModel: {err}"))
            return
        ident = envelope.get_field(msg.data, "identifier")
        if not ident:
            self.respond(msg, envelope.error("'identifier' is required"))
            return
        req = json.loads(msg.data)
        deadline = time.monotonic() + self.cfg.timeout_pull      # `nats_llm_studio.go:251` (10 min)
        try:
            res = self.store.pull(ident, deadline=deadline)
        except PullError as e:
            self.respond(msg, envelope.failure(str(e), {"model": ident, "output": e.output}))
            return
        except Exception as e:
            self.respond(msg, envelope.failure(f"failed to pull '{ident}': {e}", {"model": ident, "output": ""}))
            return
        self.registry.scan()
        data = {"model": ident, "output": res["output"], "local_paths": res["paths"],
                "bytes": res["bytes"], "seconds": round(res["seconds"], 3)}
        if req.get("load") and isinstance(self.backend, EngineBackend):
            ent = self.registry.resolve(ident) or (self.registry.resolve(os.path.basename(os.path.dirname(res["paths"][0])))
                                                   if res["paths"] else None)
            if ent is not None:
                t0 = time.time()
                try:
                    self.backend.load(ent)
                    data["loaded"] = ent.id
                    data["load_seconds"] = round(time.time() - t0, 3)
                except Exception as e:
                    data["load_error"] = str(e)
        self.respond(msg, envelope.ok(data), changed=True)

    def on_delete_model(self, msg):
        err = envelope.go_json_error(msg.data, "DeleteModelRequest", {"model_id": "ModelID"})
        if err:
            self.respond(msg, envelope.error(f"invalid JSON in DeleteModel: {err}"))
            return
        mid = envelope.get_field(msg.data, "model_id")
        if not mid:
            self.respond(msg, envelope.error("'model_id' is required"))
            return
        deadline = time.monotonic() + self.cfg.timeout_delete if self.cfg.timeout_delete > 0 else None
        self.respond(msg, self._delete(mid, deadline), changed=True)

    def _delete(self, mid: str, deadline: Optional[float]) -> bytes:
        """DeleteModel (`nats_llm_studio.go:99-133`) under the handler's 2-minute context (`:289`): the
        context bounds the unload (`:104`) and the model lookup (`:106`); the directory check and removal
        run to completion, so the reply always says what happened to the files."""
        self.registry.scan()
        ent = self.registry.resolve(mid)
        if ent is None:
            return envelope.failure(f"model not found: {mid}", {"model_id": mid, "dir": ""})
        self._unload_bounded(ent.id, deadline)             # best effort, like `lms unload` (`:87-97`)
        if deadline is not None and time.monotonic() > deadline:
            # the reference's info lookup fails on the expired context (`:106-109`): nothing is removed
            return envelope.failure("context deadline exceeded", {"model_id": mid, "dir": ""})
        d = ent.dir
        if not self.registry.safe_dir(d):
            return envelope.failure(f"refusing to delete outside MODELS_DIR: {d}", {"model_id": mid, "dir": d})
        if not os.path.isdir(d):
            return envelope.failure(f"model directory not found: {d}", {"model_id": mid, "dir": d})
        try:
            ModelStore.remove_dir(d)
        except OSError as e:
            return envelope.failure(f"error removing model directory {d}: {e}", {"model_id": mid, "dir": d})
        self.registry.scan()
        return envelope.ok({"model_id": mid, "deleted_dir": d})

    def on_chat_model(self, msg):
        t_recv = time.monotonic()
        if len(msg.data) == 0:
            self.respond(msg, envelope.error("payload vazio em ChatModel"))
            return
        err = envelope.go_json_error(msg.data, "", {"model": "Model"})
        if err:
            self.respond(msg, envelope.error(f"invalid JSON in ChatModel: {err}"))
            return
        model = envelope.get_field(msg.data, "model")
        if not model:
            self.respond(msg, envelope.error("'model' is required in ChatModel"))
            return
        req = json.loads(msg.data)
        if isinstance(self.backend, HttpBackend):           # forwards the ORIGINAL bytes (`:348`)
            try:
                status, body = self.backend.chat_raw(bytes(msg.data))
            except Exception as e:
                self.respond(msg, envelope.error(f"error calling LM Studio: {e}", {"http_status": 0}))
                return
            raw = self._raw_json(body)
            self.respond(msg, envelope.FALLBACK if raw is None else
                         envelope.ok({"http_status": status, "response": raw}))
            return
        entry = self.registry.resolve(model)
        if entry is None and isinstance(self.backend, EngineBackend):
            self.registry.scan()
            entry = self.registry.resolve(model)
        deadline = t_recv + self.cfg.timeout_chat      # from receipt (`nats_llm_studio.go:328`), JIT load included
        stream_cb = None
        ssubj = req.get("stream_subject")
        if req.get("stream") and isinstance(ssubj, str) and ssubj:
            def stream_cb(delta, _s=ssubj):
                try:
                    self.client.publish(_s, json.dumps({"object": "chat.completion.chunk", "model": model,
                                                        "choices": [{"index": 0, "delta": {"content": delta}}]}).encode())
                except Exception:
                    pass

        t_valid = time.monotonic()

        def done(status: int, body: dict, marks: dict = None):
            if status <= 0:
                self.respond(msg, envelope.error(body.get("error", "chat failed"), {"http_status": 0}))
            else:
                self.respond(msg, envelope.ok({"http_status": status, "response": body}))
            mk = {"recv": t_recv, "validated": t_valid, "responded": time.monotonic()}
            rid = ""
            for k, v in (marks or {}).items():
                if k == "request_id":
                    rid = v
                elif v:
                    mk[k] = v
            self.tracer.record("chat_model", rid or body.get("id", ""), mk,
                               {"model": model, "http_status": status})
        try:
            self.backend.chat(entry.id if entry else model, entry, req, done, deadline, stream_cb)
        except Exception as e:
            self.respond(msg, envelope.error(f"chat backend error: {e}", {"http_status": 0}))

    def on_sync_model_from_bucket(self, msg):
        try:
            req = json.loads(msg.data or b"{}")
            if not isinstance(req, dict):
                raise ValueError("request must be a JSON object")
        except Exception as e:
            self.respond(msg, envelope.error(f"invalid JSON in SyncModelFromBucket: {e}"))
            return
        missing = [k for k in ("object_name", "publisher", "model_dir") if not req.get(k)]
        if missing:
            self.respond(msg, envelope.error(f"'{missing[0]}' is required"))
            return
        bucket = req.get("bucket") or self.cfg.bucket
        try:
            res = self.store.sync(bucket, req["object_name"], req["publisher"], req["model_dir"],
                                  req.get("filename", "model.gguf"), deadline=time.monotonic() + self.cfg.timeout_pull)
        except Exception as e:
            self.respond(msg, envelope.failure(str(e), {"bucket": bucket, "object_name": req["object_name"]}))
            return
        self.registry.scan()          # the `lms import` step of README.md:305-308
        self.respond(msg, envelope.ok(res), changed=True)

    def on_metrics(self, msg):
        data = {
            "uptime_s": round(time.time() - self.t_start, 3),
            "requests": self._request_counts(),
            "latency_ms": {k: v.summary_ms() for k, v in self.latency.items()},
            "trace": self.tracer.summary(),
            "backend": self.backend.stats(),
            "nats": self.client.stats(),
            "models_dir": self.cfg.models_dir,
            "queue_group": self.cfg.queue_group,
        }
        self.respond(msg, envelope.ok(data))

    def _request_counts(self) -> dict:
        out = dict(self.counters)
        sub = next((x for x in self.subs if x.subject == self.cfg.subject("list_models")), None)
        native = sub.auto_replied if sub is not None else 0
        if native:              # answered by the native responder (no handler latency recorded for them)
            out["list_models_native"] = native
            out["list_models"] = out.get("list_models", 0) + native
        return out

    def on_health(self, msg):
        self.respond(msg, envelope.ok({"status": "ok", "pid": os.getpid(), "backend": self.backend.name,
                                       "models_loaded": self.backend.loaded_ids(),
                                       "uptime_s": round(time.time() - self.t_start, 3)}))
