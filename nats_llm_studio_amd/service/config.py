"""Worker configuration: environment (the README's variable names, `README.md:488-502`),
`.env` files (written by the reference's setup scripts, `scripts/setup_unix.sh:109-118`)
and CLI flags. The reference documents these but never reads them
(`nats_llm_studio.go:34` takes constructor args only); here they are live.
"""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass, field
from typing import Dict, Optional

SUBJECT_PREFIX = "lmstudio"


def load_dotenv(path: str = ".env", override: bool = False) -> Dict[str, str]:
    vals = {}
    if not os.path.exists(path):
        return vals
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            k, _, v = line.partition("=")
            k = k.strip()
            if k.startswith("export "):
                k = k[7:].strip()
            v = v.strip().strip('"').strip("'")
            vals[k] = v
            if override or k not in os.environ:
                os.environ[k] = v
    return vals


@dataclass
class WorkerConfig:
    nats_url: str = "nats://127.0.0.1:4222"
    models_dir: str = field(default_factory=lambda: os.path.expanduser("~/.lmstudio/models"))
    queue_group: str = "lmstudio-workers"
    subject_prefix: str = SUBJECT_PREFIX
    bucket: str = "llm-models"
    backend: str = "engine"            # engine | stub | http (proxy to an LM Studio server, the reference's mode)
    device: str = "auto"               # auto | cuda:N | cpu
    tp: int = 1                        # tensor-parallel ranks (launch with torchrun, one process per GPU)
    ep: bool = False                   # MoE: expert-parallel instead of TP-sharded experts
    model: str = ""                    # model to preload (registry id or .gguf path; required when tp > 1)
    max_batch: int = 64
    max_ctx: int = 0                   # 0 = model context length
    kv_mem_fraction: float = 0.5
    # prefill chunk: 4096 tokens (512 burst prompts: TTFT p50 417 vs 462-481 ms at 2048, profiles/service_prefill_chunk_r06.txt);
    # expert-parallel engines cap it at the EP row exchange's 2048 tokens (backends.py)
    max_prefill_tokens: int = 4096
    max_loaded_models: int = 1
    default_max_tokens: int = 512
    embedded_server: bool = False      # start an in-process NATS server at nats_url's port
    store_dir: str = ""                # JetStream persistence for the embedded server
    # per-subject handler timeouts (reference: list 30 s, pull 10 min, delete 2 min, chat 2 min)
    timeout_list: float = 30.0
    timeout_pull: float = 600.0
    timeout_delete: float = 120.0
    timeout_chat: float = 120.0
    handler_workers: int = 4
    # list_models answered by the NATS client's reader thread from the cached registry reply (kept current on every
    # reply the service sends and every list_refresh_ms): BASELINE config 1's RTT path without Python. 0 = handler
    native_list_models: bool = True
    list_refresh_ms: float = 50.0
    lmstudio_base_url: str = "http://127.0.0.1:1234"   # used by the `http` backend only
    # NATS authentication (nats.go options): token, user/password, nkey seed or a .creds file
    nats_token: str = ""
    nats_user: str = ""
    nats_password: str = ""
    nats_nkey_seed: str = ""
    nats_creds: str = ""
    # NATS TLS (nats.go: Secure / RootCAs / ClientCert / InsecureSkipVerify / TLSHandshakeFirst); a tls://
    # NATS_URL also turns it on
    nats_tls: bool = False
    nats_tls_ca: str = ""
    nats_tls_cert: str = ""
    nats_tls_key: str = ""
    nats_tls_insecure: bool = False
    nats_tls_first: bool = False

    def nats_auth(self) -> dict:
        """Keyword arguments of natsio.Client.connect for the configured credentials and TLS."""
        return dict(token=self.nats_token, user=self.nats_user, password=self.nats_password,
                    nkey_seed=self.nats_nkey_seed, creds=self.nats_creds, tls=self.nats_tls,
                    tls_ca=self.nats_tls_ca, tls_cert=self.nats_tls_cert, tls_key=self.nats_tls_key,
                    tls_insecure=self.nats_tls_insecure, tls_first=self.nats_tls_first)

    def subject(self, name: str) -> str:
        return f"{self.subject_prefix}.{name}"

    @classmethod
    def from_env(cls, env: Optional[Dict[str, str]] = None) -> "WorkerConfig":
        e = dict(os.environ if env is None else env)
        c = cls()
        c.nats_url = e.get("NATS_URL", c.nats_url)
        c.models_dir = os.path.expanduser(e.get("MODELS_DIR", e.get("LMSTUDIO_MODELS_DIR", c.models_dir)))
        c.queue_group = e.get("NATS_QUEUE_GROUP", c.queue_group)
        c.bucket = e.get("BUCKET", e.get("NATS_OBJECT_BUCKET", c.bucket))
        c.backend = e.get("BACKEND", c.backend)
        c.device = e.get("DEVICE", c.device)
        c.tp = int(e.get("TP", c.tp))
        c.ep = e.get("EP", "0") in ("1", "true", "yes")
        c.model = e.get("MODEL", c.model)
        c.max_batch = int(e.get("MAX_BATCH", c.max_batch))
        c.max_ctx = int(e.get("MAX_CTX", c.max_ctx))
        c.kv_mem_fraction = float(e.get("KV_MEM_FRACTION", c.kv_mem_fraction))
        c.max_prefill_tokens = int(e.get("MAX_PREFILL_TOKENS", c.max_prefill_tokens))
        c.lmstudio_base_url = e.get("LMSTUDIO_BASE_URL", c.lmstudio_base_url)
        c.native_list_models = e.get("NATIVE_LIST_MODELS", "1") not in ("0", "false", "no")
        c.list_refresh_ms = float(e.get("LIST_REFRESH_MS", c.list_refresh_ms))
        c.subject_prefix = e.get("SUBJECT_PREFIX", c.subject_prefix)
        c.embedded_server = e.get("EMBEDDED_NATS", "0") in ("1", "true", "yes")
        c.store_dir = e.get("NATS_STORE_DIR", c.store_dir)
        c.nats_token = e.get("NATS_TOKEN", c.nats_token)
        c.nats_user = e.get("NATS_USER", c.nats_user)
        c.nats_password = e.get("NATS_PASSWORD", c.nats_password)
        c.nats_nkey_seed = e.get("NATS_NKEY_SEED", c.nats_nkey_seed)
        seed_file = e.get("NATS_NKEY_SEED_FILE", "")
        if seed_file and not c.nats_nkey_seed:
            with open(os.path.expanduser(seed_file)) as f:
                c.nats_nkey_seed = f.read().strip()
        c.nats_creds = e.get("NATS_CREDS", c.nats_creds)
        yes = ("1", "true", "yes")
        c.nats_tls = e.get("NATS_TLS", "0").lower() in yes
        c.nats_tls_ca = e.get("NATS_TLS_CA", c.nats_tls_ca)
        c.nats_tls_cert = e.get("NATS_TLS_CERT", c.nats_tls_cert)
        c.nats_tls_key = e.get("NATS_TLS_KEY", c.nats_tls_key)
        c.nats_tls_insecure = e.get("NATS_TLS_INSECURE", "0").lower() in yes
        c.nats_tls_first = e.get("NATS_TLS_FIRST", "0").lower() in yes
        return c

    @classmethod
    def from_args(cls, argv=None) -> "WorkerConfig":
        load_dotenv(os.environ.get("DOTENV", ".env"))
        c = cls.from_env()
        ap = argparse.ArgumentParser("nats-llm-studio-amd worker")
        ap.add_argument("--nats-url", default=c.nats_url)
        ap.add_argument("--models-dir", default=c.models_dir)
        ap.add_argument("--queue-group", default=c.queue_group)
        ap.add_argument("--bucket", default=c.bucket)
        ap.add_argument("--backend", default=c.backend, choices=["engine", "stub", "http"])
        ap.add_argument("--lmstudio-base-url", default=c.lmstudio_base_url)
        ap.add_argument("--model", default=c.model)
        ap.add_argument("--ep", action="store_true", default=c.ep)
        ap.add_argument("--device", default=c.device)
        ap.add_argument("--tp", type=int, default=c.tp)
        ap.add_argument("--max-batch", type=int, default=c.max_batch)
        ap.add_argument("--max-ctx", type=int, default=c.max_ctx)
        ap.add_argument("--embedded-server", action="store_true", default=c.embedded_server)
        ap.add_argument("--store-dir", default=c.store_dir)
        ap.add_argument("--subject-prefix", default=c.subject_prefix)
        ap.add_argument("--nats-creds", default=c.nats_creds, help="NATS .creds file (user JWT + nkey seed)")
        ap.add_argument("--nats-tls-ca", default=c.nats_tls_ca, help="CA bundle for the NATS server certificate")
        ap.add_argument("--nats-tls-cert", default=c.nats_tls_cert, help="client certificate (mutual TLS)")
        ap.add_argument("--nats-tls-key", default=c.nats_tls_key, help="client key (mutual TLS)")
        a = ap.parse_args(argv)
        for k, v in vars(a).items():
            setattr(c, k, v)
        return c
