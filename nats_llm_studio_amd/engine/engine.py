"""Continuous-batching inference engine with a paged KV cache and hipGraph-captured decode.

Replaces LM Studio's request path behind `lmstudio.chat_model`
(`/root/reference/nats_llm_studio.go:327-364` -> `:158-179`), where the reference
serialises one generation per subscription. Here every in-flight request shares
each decode step:

  admission (KV blocks for the prompt only; decode grows a sequence one block at a time and, when
  the pool runs dry, preempts the most recently admitted sequences -- their blocks are freed and
  they are re-prefilled from prompt + generated tokens when room returns: recompute preemption)
   -> chunked prefill (eager; quantised GEMVs in 64-row chunks + paged attention)
   -> decode loop: one hipGraph replay per step for the padded batch bucket
      + ONE host<-device copy of the next-token ids
   -> stop checks (eos / stop ids / stop strings / max_tokens / deadline) -> Future
"""
from __future__ import annotations

import collections
import hashlib
import itertools
import os
import math
import threading
import time
from collections import defaultdict, deque
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Callable, Deque, Dict, List, Optional, Sequence as Seq

import numpy as np
import torch

from .. import ops
from ..models.llama import LlamaModel
from .sampling import HIST, SamplingParams, sample_rows, sample_rows_dev, sample_rows_gpu, uniform01

BUCKETS = (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 192, 256, 384, 512, 640, 768, 1024)

# tensor-parallel control messages (rank 0 -> followers), see Engine.follow()
_OP_STOP, _OP_PREFILL, _OP_DECODE, _OP_CAPTURE, _OP_SYNC, _OP_RESET = 0, 1, 2, 3, 4, 5
# header: op | T | nrows | need_logits | nseq | pad | candidate mode | in-graph sampling | sampling rows | 0
_HDR = 10
# NLS_TP_TRACE=1: every rank logs each control op it sends / replays (stderr), to line up the ranks' op
# sequences after a one-shot timeout
_TP_TRACE = os.environ.get("NLS_TP_TRACE", "0") == "1"
_NO_REPLAY = os.environ.get("NLS_GRAPH_NO_REPLAY", "0") == "1"
# single-GPU prefill: the first tokens of finished prompts are read back once per engine step, not per chunk
_ASYNC_FIRST = os.environ.get("NLS_ASYNC_FIRST", "1") == "1"
# single-GPU prefill of ONE prompt chunk of <= 64 tokens (a chat request's prompt): a captured graph per token bucket
# instead of ~230 eager launches, whose host time (~2.5 ms on the 8B) exceeded the GPU time
_PREFILL_GRAPHS = os.environ.get("NLS_PREFILL_GRAPHS", "1") == "1"
_NSEG = 6        # int32 step metadata segments: ids | pos | slot | tok_seq | ctx_len | use_prev (+ block tables)


@dataclass
class GenRequest:
    prompt_ids: List[int]
    params: SamplingParams = field(default_factory=SamplingParams)
    request_id: str = ""
    on_token: Optional[Callable[[int], None]] = None
    deadline: Optional[float] = None       # time.monotonic() deadline


@dataclass
class GenResult:
    request_id: str
    token_ids: List[int]
    text: str
    prompt_tokens: int
    completion_tokens: int
    finish_reason: str                     # stop | length | timeout | cancelled | error
    stop_reason: str                       # eosFound | stopStringFound | maxPredictedTokensReached | ...
    time_to_first_token: float
    generation_time: float
    error: Optional[str] = None
    t_submit: float = 0.0                  # monotonic marks for request tracing
    t_admit: float = 0.0
    t_first: float = 0.0
    t_done: float = 0.0

    @property
    def tokens_per_second(self) -> float:
        return self.completion_tokens / self.generation_time if self.generation_time > 0 else 0.0


class BlockAllocator:
    """Paged-KV block pool with automatic prefix caching.

    Full prompt blocks are content-addressed by a chained hash of their tokens (block i's key
    covers tokens [0, (i+1)*bs)), so a request whose prompt starts like an earlier one (same
    system prompt / chat history) maps those blocks read-only and prefills only the rest. Blocks
    are reference-counted; a released cached block keeps its KV and sits in an LRU until the pool
    needs it, uncached free blocks are handed out first."""

    def __init__(self, n: int, cache: bool = True):
        self.n = n
        self.cache_enabled = cache
        self.free: Deque[int] = deque(range(n))           # never-cached / invalidated blocks
        self.lru: "collections.OrderedDict[int, None]" = collections.OrderedDict()   # cached, ref 0
        self.ref = [0] * n
        self.key_of: Dict[int, bytes] = {}                 # block -> chain digest
        self.block_of: Dict[bytes, int] = {}               # chain digest -> block
        self.hits = 0                                      # prompt tokens served from the cache

    _KEY = os.urandom(16)        # per-process key: block digests cannot be precomputed by a client

    @staticmethod
    def chain_keys(tokens: Seq[int], bs: int, n_blocks: int) -> List[bytes]:
        """Keyed BLAKE2b chain over the token ids: block i's key commits to tokens [0, (i+1)*bs),
        so a cached block is reused only for the exact same prefix (no hash-collision reuse of
        another request's KV)."""
        keys, h = [], b""
        arr = np.asarray(tokens[:n_blocks * bs], dtype=np.int64)
        for i in range(n_blocks):
            h = hashlib.blake2b(h + arr[i * bs:(i + 1) * bs].tobytes(), digest_size=16,
                                key=BlockAllocator._KEY).digest()
            keys.append(h)
        return keys

    def match(self, keys: Seq[int]) -> List[int]:
        """Longest cached prefix (blocks are pinned: ref += 1)."""
        out = []
        if not self.cache_enabled:
            return out
        for k in keys:
            b = self.block_of.get(k)
            if b is None:
                break
            out.append(b)
        for b in out:
            if self.ref[b] == 0:
                self.lru.pop(b, None)
            self.ref[b] += 1
        return out

    def alloc(self, k: int) -> Optional[List[int]]:
        if k > len(self.free) + len(self.lru):
            return None
        out = []
        for _ in range(k):
            if self.free:
                b = self.free.popleft()
            else:                                           # evict the least recently used cached block
                b, _ = self.lru.popitem(last=False)
                del self.block_of[self.key_of.pop(b)]
            self.ref[b] = 1
            out.append(b)
        return out

    def register(self, blocks: Seq[int], keys: Seq[int]):
        """Publish full prompt blocks (after their KV is written) for later requests."""
        if not self.cache_enabled:
            return
        for b, k in zip(blocks, keys):
            if k not in self.block_of and b not in self.key_of:
                self.block_of[k] = b
                self.key_of[b] = k

    def release(self, blocks: Seq[int]):
        for b in blocks:
            self.ref[b] -= 1
            if self.ref[b] == 0:
                if b in self.key_of:
                    self.lru[b] = None
                else:
                    self.free.append(b)

    @property
    def n_free(self) -> int:
        return len(self.free) + len(self.lru)


class _Seq:
    __slots__ = ("req", "fut", "tokens", "n_prompt", "n_prefilled", "blocks", "t_submit", "t_admit", "t_first",
                 "t_done", "gen", "max_new", "done", "text_cache", "row", "n_fed", "keys", "n_cached", "n_target",
                 "preempted")

    def __init__(self, req: GenRequest, fut: Future):
        self.req = req
        self.fut = fut
        self.tokens = list(req.prompt_ids)
        self.n_prompt = len(req.prompt_ids)
        self.n_target = self.n_prompt   # tokens to prefill before decoding (prompt + generated after a preemption)
        self.preempted = 0
        self.n_prefilled = 0
        self.blocks: List[int] = []
        self.t_submit = time.monotonic()
        self.t_admit = None
        self.t_first = None
        self.t_done = None
        self.gen = None
        self.max_new = req.params.max_tokens
        self.done = False
        self.row = -1          # decode-batch row (stable for the sequence's life)
        self.n_fed = 0         # positions whose KV is written or being written
        self.keys: List[bytes] = []   # prefix-cache chain digests of the full prompt blocks
        self.n_cached = 0      # prompt tokens whose KV came from the prefix cache
        self.text_cache = None  # [StreamDecoder, text] of the generation (stop-string checks)

    @property
    def generated(self) -> List[int]:
        return self.tokens[self.n_prompt:]


class Engine:
    def __init__(self, model: LlamaModel, tokenizer=None, max_batch: int = 64, block_size: int = 16,
                 num_blocks: Optional[int] = None, max_prefill_tokens: int = 2048, use_graphs: bool = True,
                 ctx: Optional[int] = None, kv_mem_fraction: float = 0.5, eos_ids: Seq[int] = (),
                 prefill_attn: bool = True, async_decode: bool = True, prefix_cache: bool = True):
        self.model = model
        self.tok = tokenizer
        self.cfg = model.cfg
        self.dev = model.device
        self.bs = block_size
        self.max_batch = min(max_batch, BUCKETS[-1])
        self.ctx = min(ctx or self.cfg.ctx, self.cfg.ctx)
        self.max_blocks = math.ceil(self.ctx / block_size)
        # f16 copies of the projection weights for the large-M dense GEMM (prefill chunks, decode
        # batches >= ops.DENSE_MIN_M): NLS_DENSE_WEIGHTS=auto (default: when the copies take at most
        # 60 % of free HBM and leave the KV pool room for max_batch x ctx -- Llama-3-8B: 15 GB of 288;
        # Llama-3-70B: 140 GB of ~245 only at small batch x context (B=512 86.3 vs
        # 96.8 ms/step with mode 7; at <= 256 rows its launches keep the quantised GEMMs, tuning "d:" -1
        # entries: B=256 51.4 vs 58.4, profiles/bench_70b_mode7.txt); the rest stays for the KV pool), 1 (always),
        # 0 (never). NLS_DENSE_EXPERTS=1 adds the MoE experts (Mixtral-8x7B: 90 GB) as a second tier
        dense = os.environ.get("NLS_DENSE_WEIGHTS", "auto")
        self.dense_bytes = 0
        self.dense_policy = dense
        if self.dev.type == "cuda" and dense != "0" and hasattr(model, "expand_dense"):
            free, _ = torch.cuda.mem_get_info(self.dev)
            budget = None
            if dense != "1":
                # auto: at most 60 % of free HBM, and never so much that the KV pool (kv_mem_fraction of what is
                # left) could not hold every row of a full batch at full context -- the copies buy ~10 % of
                # large-batch step time, a squeezed pool costs admissions (Llama-3-70B at 512 x 480 tokens:
                # 79 GB of KV, no copies; Llama-3-8B: 31 GB, copies kept)
                esz = torch.finfo(getattr(model, "kv_dtype", torch.bfloat16)).bits // 8
                kv_need = (self.max_batch * self.ctx * 2 * self.cfg.n_layer * model.Hkv * model.D * esz
                           if num_blocks is None else 0)
                budget = max(0, min(int(0.60 * free), int(free - kv_need / max(kv_mem_fraction, 1e-3))))
                frac = model.dense_decode_fraction(self.max_batch) if hasattr(model, "dense_decode_fraction") else 1.0
                if frac < 0.5:
                    # decode (mostly) never takes the dense GEMMs at this batch -- below ops.DENSE_MIN_M, or the tuned
                    # "d:" entries chose the quantised GEMM: the copies would serve prompt chunks only, so they stay
                    # small next to the KV pool (Llama-3-8B: 15 GB, kept; Llama-3-70B at B <= 128: 139 GB, not -- 29.40
                    # vs 29.51 ms/step at B=128 without / with them, 241 vs 104 GB of HBM left, profiles/
                    # dense_copies_policy_r06.txt; its prefill runs on the quantised mode-9 GEMMs)
                    budget = min(budget, int(0.25 * free))
            self.dense_bytes = model.expand_dense(budget, experts=os.environ.get("NLS_DENSE_EXPERTS", "0") == "1")
            if dense != "1" and self.dense_bytes == 0:
                self.dense_policy = "auto: no copies (KV pool for max_batch x ctx first)"
        if num_blocks is None:
            # every row at full context, plus the admission watermark (below) on top: a pool sized to the
            # worst case never preempts
            num_blocks = self.max_batch * self.max_blocks
            num_blocks += num_blocks // 99 + 1
            if self.dev.type == "cuda":
                esz = torch.finfo(getattr(model, "kv_dtype", torch.bfloat16)).bits // 8
                per_block = 2 * self.cfg.n_layer * block_size * model.Hkv * model.D * esz
                free, _ = torch.cuda.mem_get_info(self.dev)
                num_blocks = int(min(num_blocks, kv_mem_fraction * free // per_block))
        self.tp = model.comm if model.shard.size > 1 else None
        self.rank = model.shard.rank
        if self.tp is not None:                # every shard must hold the same KV block pool
            num_blocks = self.tp.min_int(num_blocks)
        self.num_blocks = num_blocks
        self.kc, self.vc = model.kv_cache(num_blocks, block_size)
        self.kv_pool_bytes = 2 * self.kc.numel() * self.kc.element_size()
        self.alloc = BlockAllocator(num_blocks, cache=prefix_cache)
        # admission keeps this many blocks free for the running sequences to grow into (fewer
        # preemptions right after a burst of admissions); NLS_KV_RESERVE=full restores worst-case
        # reservation of prompt + max_tokens at admission (no growth, no preemption)
        self.watermark = max(1, num_blocks // 100)
        # preemption hysteresis: for PRESSURE_STEPS steps after a preemption, admission (new and preempted
        # sequences alike) keeps one free block per running sequence (~16 decode steps of growth for all of
        # them) instead of the 1 % watermark, so a sequence just re-admitted is not the next victim at once
        self._pressure_until = -1
        # expected-growth admission: a sequence is admitted only while the pool covers the EXPECTED blocks of
        # every running sequence plus its own -- prompt + gen_ratio * max_tokens, gen_ratio an EMA of
        # generated / max_tokens over finished requests (starts at 1: as safe as worst-case reservation until
        # requests are seen to stop early, then approaching on-demand). Preemption stays the safety net when
        # the estimate is exceeded. 512 x 1152-token requests over a 9x oversubscribed pool: on-demand alone
        # recomputed 30 % of all forward tokens (profiles/kv_pressure_r04.txt).
        self.gen_ratio = 1.0
        self.reserve_full = os.environ.get("NLS_KV_RESERVE", "ondemand") == "full"
        self.max_prefill = max_prefill_tokens
        self.prefill_attn = prefill_attn      # MFMA flash-prefill attention (else per-token decode kernel)
        self.db = model.step_buffers(self.max_batch, self.max_batch, self.max_blocks)
        self.pb = model.step_buffers(max_prefill_tokens, self.max_batch, self.max_blocks)
        pin = self.dev.type == "cuda"
        # decode metadata / next-token host buffers are double-buffered (async decode: step N+1 is
        # prepared and launched while step N's copies may still be in flight)
        self.h_meta_d2 = [torch.zeros(self.db.meta.numel(), dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.h_meta_d = self.h_meta_d2[0]
        # prefill metadata and its logit-row / query-block staging: double-buffered too. A prompt longer than
        # one chunk queues chunk after chunk with no host sync in between (no token is read back), and a
        # non_blocking copy from pinned memory reads the host buffer when it EXECUTES -- so the next chunk
        # writes the other set, after waiting on the event recorded behind this set's last uploads
        self.h_meta_p2 = [torch.zeros(self.pb.meta.numel(), dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.h_meta_p = self.h_meta_p2[0]
        self._pfk = 0
        self._first_pending: list = []          # (event, pinned ids, seqs, sampled rows): first tokens in flight
        self._first_pool: List[torch.Tensor] = []
        self._pf_ev = [torch.cuda.Event() for _ in range(2)] if pin else [None, None]
        self.h_next = torch.zeros(self.db.pad, dtype=torch.int32, pin_memory=pin)
        self.h_next2 = [torch.zeros(self.db.pad, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self._ev = [torch.cuda.Event() for _ in range(2)] if pin else [None, None]
        self._kbuf = 1
        self._inflight = None
        self.rows: List[Optional[_Seq]] = [None] * self.max_batch
        self.async_decode = async_decode
        self.use_graphs = use_graphs and self.dev.type == "cuda"
        self.graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}     # (bucket, logits needed) -> graph
        self.pf_graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}  # (token bucket, logits needed) -> prefill graph
        self.eos = set(int(e) for e in eos_ids)
        if tokenizer is not None and getattr(tokenizer, "eos_id", None) is not None:
            self.eos.add(int(tokenizer.eos_id))
        if tokenizer is not None:
            for name in ("<|eot_id|>", "<|end_of_text|>", "<|eom_id|>", "</s>", "<|im_end|>", "<|endoftext|>"):
                tid = tokenizer.vocab.get(name) if hasattr(tokenizer, "vocab") else None
                if tid is not None:
                    self.eos.add(int(tid))
        self.waiting: Deque[_Seq] = deque()
        self.running: List[_Seq] = []
        self.lock = threading.Condition()
        self.thread: Optional[threading.Thread] = None
        self.stop_flag = False
        self._ids = itertools.count()
        self.host_ms = defaultdict(float)
        self.counters = dict(steps=0, decode_tokens=0, prefill_tokens=0, requests=0, graph_replays=0,
                             prefill_graph_replays=0,
                             device_sampled_steps=0, preemptions=0, recompute_tokens=0, candidate_sampled_steps=0,
                             candidate_sampled_prefills=0)
        self.full_logits: Optional[torch.Tensor] = None
        # TP sampling: per-rank top-CAND candidates gathered instead of the full logits when every sampled row
        # of the step has 0 < top_k <= CAND - HIST (or samples at temperature 0 with penalties); see _cand_ok
        self.cand: Optional[tuple] = None
        self._cand_mode = False
        self._ctrl_hdr = torch.zeros(_HDR + self.max_batch, dtype=torch.int32)
        # In-graph sampling: per-row sampling params / seeds / penalty-history rings live on the device,
        # written once when a sequence takes its decode row; sampled rows then stay on the chained
        # asynchronous decode path (ops.sample_decode after the lm-head, inside the hipGraph). Tensor
        # parallel: every rank holds the same rows (shipped with the step's control message), gathers the
        # per-rank top-CAND candidates through the IPC one-shot kernel and runs the same draw
        # (ops.sample_decode_cand), so the sampled ids agree on every rank with no host round trip. Needs
        # the one-shot data plane on GPUs (an RCCL gather would put RCCL back into the graph); the CPU gloo
        # rehearsal runs the same sequence eagerly.
        oneshot_ = getattr(model.comm, "oneshot", None) if self.tp is not None else None
        self.device_sampling = (os.environ.get("NLS_DEVICE_SAMPLING", "1") == "1" and (
            (self.dev.type == "cuda" and self.tp is None)
            or (self.tp is not None and (self.dev.type == "cpu" or oneshot_ is not None))))
        if self.device_sampling:
            self.d_sparams = torch.zeros(self.max_batch, ops.SAMPLE_PARAMS_BYTES, dtype=torch.uint8, device=self.dev)
            self.d_seeds = torch.zeros(self.max_batch, dtype=torch.int64, device=self.dev)
            self.d_hist = torch.full((self.max_batch, HIST), -1, dtype=torch.int32, device=self.dev)
            # rows taking a decode slot are staged in pinned memory (double-buffered like the step
            # metadata) and go up as ONE async copy + device scatter before the next launch: per-row
            # pageable copies stall the host and serialise behind the step in flight (a 512-request
            # burst paid ~1.5K of them)
            nb_ = ops.SAMPLE_PARAMS_BYTES
            self._srow_pin = [dict(idx=torch.zeros(self.max_batch, dtype=torch.int64, pin_memory=pin),
                                   par=torch.zeros(self.max_batch, nb_, dtype=torch.uint8, pin_memory=pin),
                                   seed=torch.zeros(self.max_batch, dtype=torch.int64, pin_memory=pin),
                                   hist=torch.zeros(self.max_batch, HIST, dtype=torch.int32, pin_memory=pin))
                              for _ in range(2)]
            self._srow_dev = dict(idx=torch.zeros(self.max_batch, dtype=torch.int64, device=self.dev),
                                  par=torch.zeros(self.max_batch, nb_, dtype=torch.uint8, device=self.dev),
                                  seed=torch.zeros(self.max_batch, dtype=torch.int64, device=self.dev),
                                  hist=torch.zeros(self.max_batch, HIST, dtype=torch.int32, device=self.dev))
            self._srow_dirty: Dict[int, tuple] = {}
        self.sync_hook: Optional[Callable[[], None]] = None   # follower side of Engine.sync()
        # tensor parallel with the IPC one-shot all-reduce: its error words (raised on every rank when any
        # rank's poll timed out) travel to the host with each step's tokens; a raised word fails the step
        self._oneshot = getattr(model.comm, "oneshot", None) if self.tp is not None else None
        self.h_err2 = ([torch.zeros(self._oneshot.ERR_WORDS, dtype=torch.int32, pin_memory=True) for _ in range(2)]
                       if self._oneshot is not None else None)

    # ------------------------------------------------------------------ API
    def submit(self, req: GenRequest) -> Future:
        fut: Future = Future()
        if not req.request_id:
            req.request_id = f"req-{next(self._ids)}"
        s = _Seq(req, fut)
        if s.n_prompt == 0:
            fut.set_exception(ValueError("empty prompt"))
            return fut
        if s.n_prompt >= self.ctx:
            fut.set_exception(ValueError(f"prompt ({s.n_prompt} tokens) exceeds the context length ({self.ctx})"))
            return fut
        # a sequence must fit the context and, alone, the whole KV pool (it can always finish once every
        # other sequence has been preempted)
        cap = min(self.ctx, self.num_blocks * self.bs)
        if s.n_prompt >= cap:
            fut.set_exception(ValueError(f"prompt ({s.n_prompt} tokens) exceeds the KV cache ({cap} tokens)"))
            return fut
        s.max_new = max(1, min(req.params.max_tokens, cap - s.n_prompt))
        if not req.params.greedy:             # one seed per request: u = uniform01(seed, position)
            sd = req.params.seed
            s.gen = (int(sd) if sd is not None else int.from_bytes(os.urandom(8), "little") >> 1) & 0x7FFFFFFFFFFFFFFF
        with self.lock:
            if self.stop_flag or self.model is None:    # unloaded / shut down: never park a request
                fut.set_exception(RuntimeError("engine is not running (model unloaded)"))
                return fut
            self.waiting.append(s)
            self.counters["requests"] += 1
            self.lock.notify_all()
        return fut

    def generate(self, prompt_ids: List[int], params: SamplingParams = None, timeout: float = None) -> GenResult:
        fut = self.submit(GenRequest(list(prompt_ids), params or SamplingParams()))
        if self.thread is None:
            while not fut.done():
                self.step()
        return fut.result(timeout)

    def start(self):
        if self.thread is None:
            self.stop_flag = False
            self.thread = threading.Thread(target=self._loop, name="nls-engine", daemon=True)
            self.thread.start()
        return self

    def shutdown(self):
        with self.lock:
            self.stop_flag = True
            self.lock.notify_all()
        if self.thread is not None:
            self.thread.join()
            self.thread = None
        try:
            self._drain()
        except Exception:
            pass
        self.stop_followers()
        for s in list(self.running) + list(self.waiting):
            self._finish(s, "cancelled", "engineShutdown")
        self.running.clear()
        self.waiting.clear()

    def unload(self):
        """Free device memory (KV cache, graphs, weights).

        May be reached from the engine thread itself (a request's completion callback releasing the
        last reference of an evicted model): then the loop is told to stop and the teardown runs on
        a helper thread once the loop has returned, never by joining the current thread."""
        if self.thread is not None and threading.current_thread() is self.thread:
            with self.lock:
                self.stop_flag = True
                self.lock.notify_all()
            threading.Thread(target=self.unload, name="nls-engine-unload", daemon=True).start()
            return
        self.shutdown()
        self.graphs.clear()
        self.pf_graphs.clear()
        self.kc = self.vc = None
        self.db = self.pb = None
        self.model = None
        if self.dev.type == "cuda":
            torch.cuda.empty_cache()

    def _loop(self):
        while True:
            with self.lock:
                while not self.stop_flag and not self.waiting and not self.running:
                    self.lock.wait(0.5)
                if self.stop_flag:
                    return
            try:
                self.step()
            except Exception as e:  # fail every in-flight request rather than hang them
                import traceback
                traceback.print_exc()
                for s in list(self.running):
                    self._finish(s, "error", "engineError", error=str(e))
                self.running.clear()
                self._inflight = None          # the failed step's tokens are discarded with its requests
                self._release_rows()

    # ------------------------------------------------------------------ scheduling
    def step(self):
        # host-time accounting (ms, cumulative; stats()["host_ms"]): where the engine thread spends a step
        # -- "wait" is blocked on the GPU (the step in flight), everything else is host work that the
        # async decode pipeline has to hide behind the GPU step
        hm, clk = self.host_ms, time.perf_counter
        t0 = clk()
        self._expire()
        self._admit()
        t1 = clk()
        hm["schedule"] += (t1 - t0) * 1e3
        # the prefill chunk is queued behind the in-flight decode step (separate step buffers) and the next
        # decode step still chains on that step's device-side tokens: no pipeline drain. With a deep prompt
        # backlog (a burst of arrivals) up to PREFILL_CHUNKS chunks run before the next decode step: fewer
        # small decode steps while the batch ramps up, earlier first tokens (NLS_PREFILL_CHUNKS)
        for c in range(self.PREFILL_CHUNKS):
            if not any(s.n_prefilled < s.n_target for s in self.running):
                break
            if c:
                self._admit()
            self._prefill()
        self._flush_first_tokens()
        t2 = clk()
        hm["prefill"] += (t2 - t1) * 1e3
        dec = [s for s in self.running if s.n_prefilled >= s.n_target and not s.done]
        if dec:
            self._decode(dec)
        else:
            self._drain()
        self.running = [s for s in self.running if not s.done]
        self.counters["steps"] += 1
        hm["decode"] += (clk() - t2) * 1e3

    def _expire(self):
        now = time.monotonic()
        for s in list(self.running):
            if s.req.deadline is not None and now > s.req.deadline:
                self._finish(s, "timeout", "timeout")
        with self.lock:
            keep = deque()
            for s in self.waiting:
                if s.req.deadline is not None and now > s.req.deadline:
                    self._finish(s, "timeout", "timeout")
                else:
                    keep.append(s)
            self.waiting = keep
        self.running = [s for s in self.running if not s.done]

    def _expected_blocks(self, s: _Seq) -> int:
        """Blocks s is expected to hold at its end: all its tokens so far + gen_ratio of what it may still
        generate (the context caps it)."""
        gen = len(s.tokens) - s.n_prompt
        rest = max(0.0, self.gen_ratio * s.max_new - gen)
        return math.ceil(min(self.ctx, s.n_target + max(0, len(s.tokens) - s.n_target) + rest) / self.bs)

    def _admit(self):
        with self.lock:
            growth = None                     # expected further blocks of the running sequences
            while self.waiting and len(self.running) < self.max_batch:
                s = self.waiting[0]
                if not self.reserve_full and self.running:
                    if growth is None:
                        growth = sum(max(0, self._expected_blocks(x) - len(x.blocks)) for x in self.running)
                    if growth + self._expected_blocks(s) > self.alloc.n_free:
                        break
                if self.reserve_full:
                    need = math.ceil((s.n_prompt + s.max_new) / self.bs)
                else:                          # the prompt now, decode blocks on demand (_ensure_blocks)
                    need = math.ceil(s.n_target / self.bs)
                # full prompt blocks, leaving >= 1 prompt token to prefill (its logits pick token 1)
                s.keys = BlockAllocator.chain_keys(s.tokens, self.bs, (s.n_target - 1) // self.bs)
                hit = self.alloc.match(s.keys)
                reserve = self.watermark if (self.running and not self.reserve_full) else 0
                if self.running and self.counters["steps"] < self._pressure_until:
                    reserve = max(reserve, len(self.running))
                blocks = None
                if need - len(hit) + reserve <= self.alloc.n_free:
                    blocks = self.alloc.alloc(need - len(hit))
                if blocks is None:
                    self.alloc.release(hit)
                    break
                s.blocks = hit + blocks
                s.n_prefilled = s.n_cached = len(hit) * self.bs
                self.alloc.hits += s.n_cached
                s.t_admit = time.monotonic()
                self.waiting.popleft()
                self.running.append(s)
                if growth is not None:
                    growth += max(0, self._expected_blocks(s) - len(s.blocks))

    def _slot(self, s: _Seq, p: int) -> int:
        return s.blocks[p // self.bs] * self.bs + p % self.bs

    def _next_prefill_buf(self):
        """Switch to the other prefill staging set once the uploads that last read it have executed."""
        self._pfk ^= 1
        ev = self._pf_ev[self._pfk]
        if ev is not None:
            ev.synchronize()
        self.h_meta_p = self.h_meta_p2[self._pfk]

    def _prefill(self):
        self._next_prefill_buf()
        b, pad = self.pb, self.pb.pad
        h = self.h_meta_p.numpy()
        ids, pos, slot, tseq, ctxl = (h[i * pad:(i + 1) * pad] for i in range(5))
        h[5 * pad:6 * pad] = 0                              # use_prev: prefill feeds host ids
        bt = h[_NSEG * pad:].reshape(self.max_batch, self.max_blocks)
        budget = self.max_prefill
        T = 0
        rows, finishing = [], []
        batch = [s for s in self.running if s.n_prefilled < s.n_target]
        for si, s in enumerate(batch):
            if budget <= 0:
                break
            n = min(budget, s.n_target - s.n_prefilled)
            p0 = s.n_prefilled
            ids[T:T + n] = s.tokens[p0:p0 + n]
            pr = np.arange(p0, p0 + n)
            pos[T:T + n] = pr
            blk = np.asarray(s.blocks, dtype=np.int64)
            slot[T:T + n] = blk[pr // self.bs] * self.bs + pr % self.bs
            tseq[T:T + n] = si
            ctxl[T:T + n] = pr + 1
            bt[si, :len(s.blocks)] = s.blocks
            s.n_prefilled += n
            T += n
            budget -= n
            if s.n_prefilled >= s.n_target:
                rows.append(T - 1)
                finishing.append(s)
                self.alloc.register(s.blocks[:len(s.keys)], s.keys)
        nrows = max(1, len(rows))
        need = any(not s.req.params.greedy for s in finishing)
        self._cand_mode = need and self._cand_ok(finishing)
        self._ctrl(_OP_PREFILL, T, nrows, need, rows + [0] * (nrows - len(rows)), len(batch), self.h_meta_p, pad)
        self._exec_prefill(T, rows + [0] * (nrows - len(rows)), need)
        self.counters["prefill_tokens"] += T
        if finishing:
            if self.dev.type == "cuda" and self.tp is None and _ASYNC_FIRST:
                self._pick_async(finishing, b)
            else:
                self._first_tokens(finishing, self._pick(finishing, b, list(range(len(finishing)))))

    def _first_tokens(self, seqs: List[_Seq], toks: List[int]):
        now = time.monotonic()
        for s, t in zip(seqs, toks):
            if s.done:                         # finished meanwhile (deadline, failed step): nothing to append
                continue
            if s.t_first is None:
                s.t_first = now
            self._append(s, t)

    def _pick_async(self, seqs: List[_Seq], b):
        """_pick without waiting for the chunk: the greedy ids and the device sampler's draws of the sequences
        whose prefill ended in this chunk are copied to a pinned buffer behind an event, and
        _flush_first_tokens appends them once per engine step, before its decode step. Back-to-back prefill
        chunks then queue with no host sync between them (each sync left the GPU idle while the host built
        and launched the next chunk)."""
        n, mb = len(seqs), self.max_batch
        if not self._first_pool:
            self._first_pool.append(torch.empty(2 * mb, dtype=torch.int32, pin_memory=True))
        pin = self._first_pool.pop()
        pin[:n].copy_(b.next_ids[:n], non_blocking=True)
        sampled = [i for i, s in enumerate(seqs) if not s.req.params.greedy]
        if sampled:
            idx = torch.tensor(sampled, dtype=torch.long).pin_memory().to(self.dev, non_blocking=True)
            toks = sample_rows_dev(b.logits.index_select(0, idx), [seqs[i].req.params for i in sampled],
                                   [seqs[i].tokens for i in sampled], [self._u(seqs[i]) for i in sampled])
            pin[mb:mb + len(sampled)].copy_(toks, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._first_pending.append((ev, pin, seqs, sampled))

    def _flush_first_tokens(self):
        pend, self._first_pending = self._first_pending, []
        mb = self.max_batch
        for ev, pin, seqs, sampled in pend:
            ev.synchronize()
            toks = pin[:len(seqs)].tolist()
            for i, t in zip(sampled, pin[mb:mb + len(sampled)].tolist()):
                toks[i] = t
            self._first_tokens(seqs, toks)
            self._first_pool.append(pin)

    PREFILL_GRAPH_T = (16, 32, 64)      # token buckets of the captured single-prompt prefill graphs

    def _pf_buffers(self):
        """Pinned staging (two sets) and the device copies of the prefill logit rows and query blocks."""
        if not hasattr(self, "_pf_pin"):
            cuda = self.dev.type == "cuda"
            nq = (self.max_prefill + 15) // 16 + self.max_batch
            self._pf_pin = [(torch.zeros(self.max_batch, dtype=torch.int32, pin_memory=cuda),
                             torch.zeros(nq, 4, dtype=torch.int32, pin_memory=cuda)) for _ in range(2)]
            self._pf_dev = (torch.zeros(self.max_batch, dtype=torch.int32, device=self.dev),
                            torch.zeros(nq, 4, dtype=torch.int32, device=self.dev))

    def _pf_graph_key(self, T: int, rows: List[int], qb, need_logits: bool):
        """The prefill graph of this chunk, if any: single GPU, one contiguous run of <= 64 tokens of one
        sequence (one query block, one logit row) -- the shape of a chat request's prompt."""
        if not (self.use_graphs and _PREFILL_GRAPHS and self.tp is None and qb is not None and len(qb) == 1
                and len(rows) == 1 and self.model.cfg.n_expert == 0):
            return None
        for Tb in self.PREFILL_GRAPH_T:
            if T <= Tb <= self.max_prefill:
                return (Tb, bool(need_logits))
        return None

    def _pf_forward(self, Tb: int, need_logits: bool):
        ld, qd = self._pf_dev
        return self.model.forward(self.pb, self.kc, self.vc, Tb, self.bs, LlamaModel.attn_splits(Tb, self.model.Hkv),
                                  logit_rows=ld[:1], n_logits=1, qblocks=qd[:1], nqb=1, need_logits=need_logits)

    def _capture_prefill(self, key):
        """Capture the prefill graph `key` on the current metadata (the caller ran the same forward eagerly)."""
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._pf_forward(*key)
        torch.cuda.synchronize(self.dev)
        self.pf_graphs[key] = g

    def _exec_prefill(self, T: int, rows: List[int], need_logits: bool):
        b = self.pb
        cuda = self.dev.type == "cuda"
        pad = b.pad
        h = self.h_meta_p.numpy()
        qb = ops.prefill_blocks(h[3 * pad:4 * pad], h[pad:2 * pad], T) if self.prefill_attn else None
        key = self._pf_graph_key(T, rows, qb, need_logits)
        if key is not None:
            # rows T .. Tb-1 of the token bucket: no KV writes (slot -1), position 0 (the RoPE table), no attention
            # (the one query block covers [0, T)); their GEMV rows compute on stale activations and are never read
            Tb = key[0]
            for seg, v in ((0, 0), (1, 0), (2, -1), (3, 0), (4, 0)):
                h[seg * pad + T:seg * pad + Tb] = v
        b.meta.copy_(self.h_meta_p, non_blocking=cuda and self.rank == 0)
        # logit rows and query blocks through pinned staging (async, stream-ordered: pageable uploads block
        # the host until the decode step in flight has drained), one set per prefill metadata buffer
        self._pf_buffers()
        # (set _pfk's previous uploads have executed: _next_prefill_buf waited on their event)
        lp, qp = self._pf_pin[self._pfk]
        ld, qd = self._pf_dev
        lp.numpy()[:len(rows)] = rows
        lr = ld[:len(rows)]
        lr.copy_(lp[:len(rows)], non_blocking=cuda)
        qbt = None
        if qb is not None and len(qb):
            if len(qb) > qp.shape[0]:
                qbt = torch.from_numpy(qb).to(self.dev)
            else:
                qp.numpy()[:len(qb)] = qb
                qbt = qd[:len(qb)]
                qbt.copy_(qp[:len(qb)], non_blocking=cuda)
        if self._pf_ev[self._pfk] is not None:
            self._pf_ev[self._pfk].record()
        if key is not None:
            g = self.pf_graphs.get(key)
            if g is not None:
                g.replay()
                self.counters["prefill_graph_replays"] += 1
                n = 1
            else:                       # first chunk of this bucket: run it eagerly, then capture for the next
                n = self._pf_forward(*key)
                self._capture_prefill(key)
        else:
            n = self.model.forward(b, self.kc, self.vc, T, self.bs, LlamaModel.attn_splits(T, self.model.Hkv),
                                   logit_rows=lr, n_logits=len(rows), qblocks=qbt, nqb=0 if qbt is None else len(qb),
                                   need_logits=need_logits)
        self._gather(b, n, need_logits)

    CAND = 128           # TP sampling: candidates per rank and row
    PREFILL_CHUNKS = int(os.environ.get("NLS_PREFILL_CHUNKS", "4"))   # prefill chunks per step (backlog)
    PRESSURE_STEPS = 64  # preemption hysteresis window (steps), see _pressure_until

    def _cand_ok(self, seqs) -> bool:
        """Can every sampled row of these sequences be drawn exactly from the gathered top-CAND candidates of
        each rank? Penalties only lower logits of the <= HIST history tokens, so the post-penalty top-k lies in
        the pre-penalty top-(k + HIST) of the vocabulary, and top-p / min-p act on the kept top-k set (the
        sampler's order): exact for 0 < top_k <= CAND - HIST, and for penalised temperature-0 rows."""
        if self.tp is None or os.environ.get("NLS_TP_CANDIDATES", "1") != "1":
            return False
        for s in seqs:
            p = s.req.params
            if p.greedy:
                continue
            # a repeat penalty < 1 or a negative presence / frequency penalty RAISES history logits: a history
            # token outside every rank's candidates could then enter the kept set -- not exact, full logits
            if p.repeat_penalty < 1.0 or p.presence_penalty < 0.0 or p.frequency_penalty < 0.0:
                return False
            if p.temperature > 0.0 and not (0 < (p.top_k or 0) <= self.CAND - HIST):
                return False
        return True

    def _gather(self, b, n: int, need_logits: bool):
        self.cand = None
        if self.tp is not None and need_logits and self._cand_mode:
            m = self.model
            valid = max(0, min(m.vocab_hi, m.cfg.vocab) - m.vocab_lo)
            self.cand = self.tp.gather_candidates(*ops.topc_candidates(b.logits, n, self.CAND, m.vocab_lo, valid))
            self.full_logits = None
        elif self.tp is not None and need_logits:
            m = self.model
            self.full_logits = self.tp.gather_logits(b.logits, n, m.cfg.vocab, m.vocab_per)
        else:
            self.full_logits = None

    # ------------------------------------------------------------------ tensor parallel control
    def _ctrl(self, op: int, T: int, nrows: int, need: bool, rows: List[int], nseq: int, hmeta: torch.Tensor,
              pad: int, dsamp: bool = False, srows: Optional[list] = None):
        """Rank 0: broadcast the step (header + used part of the packed metadata + the sampling rows that
        took a decode row since the last step) to followers."""
        if self.tp is None:
            return
        nb = self.max_blocks
        hdr = self._ctrl_hdr
        hdr.zero_()
        hdr[:_HDR] = torch.tensor([op, T, nrows, int(need), nseq, pad, int(self._cand_mode), int(dsamp),
                                   len(srows or ()), 0], dtype=torch.int32)
        if rows:
            hdr[_HDR:_HDR + len(rows)] = torch.tensor(rows, dtype=torch.int32)
        self.tp.bcast_ctrl(hdr)
        if _TP_TRACE:
            self._trace_op("send", hdr)
        if op in (_OP_PREFILL, _OP_DECODE):
            self.tp.bcast_ctrl(hmeta[:_NSEG * pad + nseq * nb].clone())
        if srows:
            self.tp.bcast_ctrl(self._pack_srows(srows))

    def _trace_op(self, what: str, hdr: torch.Tensor):
        import sys
        self._nops = getattr(self, "_nops", 0) + 1
        print(f"[tp r{self.rank}] {time.monotonic():.6f} #{self._nops} {what} " + " ".join(str(int(v)) for v in hdr[:9]),
              file=sys.stderr, flush=True)

    _SROW = 1 + ops.SAMPLE_PARAMS_BYTES // 4 + 2 + HIST     # int32 words of one shipped sampling row

    @staticmethod
    def _pack_srows(srows) -> torch.Tensor:
        out = np.zeros((len(srows), Engine._SROW), dtype=np.int32)
        for i, (r, raw, seed, hist) in enumerate(srows):
            out[i, 0] = r
            o = 1 + ops.SAMPLE_PARAMS_BYTES // 4
            out[i, 1:o] = np.frombuffer(raw, dtype=np.int32)
            out[i, o:o + 2] = np.array([seed], dtype=np.int64).view(np.int32)
            out[i, o + 2:] = hist
        return torch.from_numpy(out.reshape(-1))

    @staticmethod
    def _unpack_srows(buf: torch.Tensor) -> list:
        a = buf.numpy().reshape(-1, Engine._SROW)
        o = 1 + ops.SAMPLE_PARAMS_BYTES // 4
        return [(int(x[0]), x[1:o].tobytes(), int(x[o:o + 2].view(np.int64)[0]), x[o + 2:].copy()) for x in a]

    def sync(self, hook: Callable[[], None]):
        """Rank 0: make every follower run its `sync_hook` now, then run `hook` here (used by the
        benchmark to bracket a timed region with a world-wide barrier while followers replay)."""
        self._drain()
        self._ctrl(_OP_SYNC, 0, 0, False, [], 0, None, 0)
        hook()

    def stop_followers(self):
        if self.tp is not None and self.rank == 0 and not getattr(self, "_followers_stopped", False):
            self._followers_stopped = True
            self._ctrl(_OP_STOP, 0, 0, False, [], 0, None, 0)

    def follow(self):
        """Follower rank main loop: replay every step rank 0 schedules until it sends STOP."""
        assert self.tp is not None and self.rank != 0
        nb = self.max_blocks
        while True:
            hdr = self.tp.bcast_ctrl(self._ctrl_hdr)
            if _TP_TRACE:
                self._trace_op("recv", hdr)
            op, T, nrows, need, nseq, pad, cand, dsamp, nsr = (int(v) for v in hdr[:9])
            self._cand_mode = bool(cand)
            if op == _OP_STOP:
                return
            if op == _OP_CAPTURE:
                self._capture(T, LlamaModel.attn_splits(T, self.model.Hkv), dsamp=bool(dsamp))
                continue
            if op == _OP_RESET:
                if _TP_TRACE:
                    import sys
                    print(f"[tp r{self.rank}] state {self._oneshot.debug_state()}", file=sys.stderr, flush=True)
                from ..ops import _lib as _oplib
                if _oplib._OP_TIMING:    # NLS_OP_TIMING: launches whose completion lagged the previous one's
                    print(f"[tp r{self.rank}] op gaps {_oplib.op_timing(50.0)}", file=sys.stderr, flush=True)
                self._oneshot.reset()
                continue
            if op == _OP_SYNC:
                if self.sync_hook is not None:
                    self.sync_hook()
                continue
            if op == _OP_PREFILL:
                self._next_prefill_buf()
            hm = self.h_meta_p if op == _OP_PREFILL else self.h_meta_d
            buf = torch.zeros(_NSEG * pad + nseq * nb, dtype=torch.int32)
            self.tp.bcast_ctrl(buf)
            hm[:buf.numel()] = buf
            if nsr:
                sb = torch.zeros(nsr * self._SROW, dtype=torch.int32)
                self.tp.bcast_ctrl(sb)
                for r, raw, seed, hist in self._unpack_srows(sb):
                    self._srow_dirty[r] = (raw, seed, hist)
            if op == _OP_PREFILL:
                self._exec_prefill(T, [int(v) for v in hdr[_HDR:_HDR + nrows]], bool(need))
            else:
                if self.device_sampling:
                    self._kbuf ^= 1
                    self._flush_sampling_rows(self._kbuf)
                self.db.meta.copy_(hm)
                self._run_decode(T, bool(need), bool(dsamp))
                if dsamp:
                    self.counters["device_sampled_steps"] += 1
                if need:
                    self._gather(self.db, T, True)

    def _pick(self, seqs: List[_Seq], b, rows: List[int]) -> List[int]:
        greedy = b.next_ids[:len(rows)].cpu().tolist() if self.dev.type != "cuda" else None
        if greedy is None:
            self.h_next[:len(rows)].copy_(b.next_ids[:len(rows)])
            greedy = self.h_next[:len(rows)].tolist()
        out = list(greedy)
        sampled = [i for i, s in enumerate(seqs) if not s.req.params.greedy]
        if sampled and self.cand is not None:
            toks = self._sample_candidates([rows[i] for i in sampled], [seqs[i] for i in sampled], prefill=True)
            for i, t in zip(sampled, toks):
                out[i] = t
            sampled = []
        if sampled:
            lg = self.full_logits if self.full_logits is not None else b.logits
            fn = sample_rows_gpu if lg.is_cuda else sample_rows
            toks = fn(lg[[rows[i] for i in sampled]], [seqs[i].req.params for i in sampled],
                      [seqs[i].tokens for i in sampled], [self._u(seqs[i]) for i in sampled])
            for i, t in zip(sampled, toks):
                out[i] = t
        return out

    def _sample_candidates(self, rows: List[int], seqs: List[_Seq], prefill: bool = False) -> List[int]:
        """Draw the sampled rows from the gathered candidates (values in vocabulary order, global ids): the
        sampler runs on the candidate rows with each history token mapped to its candidate position (history
        tokens outside the candidates cannot reach the kept set); the drawn position maps back to its id.
        Same kept set, same index order, same variate: the token the full-vocabulary sampler would draw."""
        vals, ids = self.cand
        # host-driven draws: the first token of sampled requests (after their prefill), and decode steps whose
        # sampled rows could not stay in the graph
        self.counters["candidate_sampled_prefills" if prefill else "candidate_sampled_steps"] += 1
        v = vals[rows]
        ix = ids[rows]
        ixl = ix.cpu().tolist()
        hist = []
        for r, s in enumerate(seqs):
            pos = {t: j for j, t in enumerate(ixl[r]) if t >= 0}
            hist.append([pos[t] for t in s.tokens[-HIST:] if t in pos])
        fn = sample_rows_gpu if v.is_cuda else sample_rows
        picks = fn(v.contiguous(), [s.req.params for s in seqs], hist, [self._u(s) for s in seqs])
        return [int(ixl[r][j]) if 0 <= j < len(ixl[r]) and ixl[r][j] >= 0 else 0 for r, j in enumerate(picks)]

    @staticmethod
    def _u(s: _Seq) -> float:
        """The variate of s's next draw: uniform01(seed, position of its last token) -- what the in-graph
        sampler uses for the same row and step."""
        return uniform01(s.gen, len(s.tokens) - 1)

    def _bucket(self, B: int) -> int:
        for k in BUCKETS:
            if k >= B and k <= self.max_batch:
                return k
        return self.max_batch

    # ------------------------------------------------------------------ decode
    # Rows: a decoding sequence keeps one row of the decode batch (and its block-table row) for
    # its whole life, so consecutive steps can chain on the device: with `use_prev` set, a row's
    # input token is the previous step's next_ids entry (written by the previous graph replay),
    # and the host can launch step N+1 before it has read step N's tokens (async decode). The
    # host then digests step N (stop checks, callbacks) while the GPU runs step N+1. A sequence
    # that stops on EOS / stop strings at step N runs one discarded step inside its own KV
    # reservation; sequences that will hit max_tokens are never launched past their budget.
    def _free_row(self) -> int:
        for i, s in enumerate(self.rows):
            if s is None:
                return i
        raise RuntimeError("no free decode row")

    def _assign_row(self, s: _Seq):
        r = self._free_row()
        self.rows[r] = s
        s.row = r
        s.n_fed = len(s.tokens) - 1
        nb = len(s.blocks)
        for hm in self.h_meta_d2:
            bt = hm.numpy()[_NSEG * self.db.pad:].reshape(self.max_batch, self.max_blocks)
            bt[r, :nb] = s.blocks
            bt[r, nb:] = 0
        if self.device_sampling:
            self._upload_sampling_row(r, s)

    def _upload_sampling_row(self, r: int, s: _Seq):
        """Row r's sampling state on the device: params (greedy rows: temperature 0, neutral penalties,
        skipped by the sampler), seed, and the last HIST tokens at ring slots (position % HIST)."""
        p = s.req.params
        if p.greedy:
            raw = ops.sample_params_bytes()
            seed = 0
        else:
            raw = ops.sample_params_bytes(p)
            seed = s.gen
        hist = np.full(HIST, -1, dtype=np.int32)
        n = len(s.tokens)
        for q in range(max(0, n - HIST), n):
            hist[q % HIST] = s.tokens[q]
        self._srow_dirty[r] = (raw, seed & 0x7FFFFFFFFFFFFFFF, hist)

    def _flush_sampling_rows(self, k: int):
        """Upload the staged rows (pinned buffer k) before the launch that first samples them: one async
        copy per table into device staging, then an index_copy_ scatter -- all ordered on the stream."""
        if not self._srow_dirty:
            return
        rows = sorted(self._srow_dirty)
        n = len(rows)
        hp, dv = self._srow_pin[k], self._srow_dev
        ip, pp, sp, hh = hp["idx"].numpy(), hp["par"].numpy(), hp["seed"].numpy(), hp["hist"].numpy()
        for j, r in enumerate(rows):
            raw, seed, hist = self._srow_dirty[r]
            ip[j] = r
            pp[j] = np.frombuffer(raw, dtype=np.uint8)
            sp[j] = seed
            hh[j] = hist
        self._srow_dirty.clear()
        for key in ("idx", "par", "seed", "hist"):
            dv[key][:n].copy_(hp[key][:n], non_blocking=True)
        idx = dv["idx"][:n]
        self.d_sparams.index_copy_(0, idx, dv["par"][:n])
        self.d_seeds.index_copy_(0, idx, dv["seed"][:n])
        self.d_hist.index_copy_(0, idx, dv["hist"][:n])

    def _release_rows(self, keep=()):
        keep = set(id(x) for x in keep)
        for i, s in enumerate(self.rows):
            if s is not None and s.done and id(s) not in keep:
                self.rows[i] = None
                s.row = -1

    def _compact(self, seqs: List[_Seq]):
        """Re-pack rows 0..n-1 (only with no step in flight: moved rows get host-side ids)."""
        for i in range(len(self.rows)):
            self.rows[i] = None
        for s in seqs:
            s.row = -1
        for s in sorted(seqs, key=lambda x: x.t_submit):
            self._assign_row(s)

    def _build_meta(self, k: int, launch: List[_Seq], prev: set) -> int:
        """Fill pinned meta buffer k for the rows of `launch`; returns the padded bucket."""
        pad = self.db.pad
        h = self.h_meta_d2[k].numpy()
        ids, pos, slot, tseq, ctxl, usep = (h[i * pad:(i + 1) * pad] for i in range(_NSEG))
        bt = h[_NSEG * pad:].reshape(self.max_batch, self.max_blocks)
        top = max(s.row for s in launch) + 1
        Bp = self._bucket(top)
        ids[:Bp] = 0
        pos[:Bp] = 0
        slot[:Bp] = -1
        ctxl[:Bp] = 0
        usep[:Bp] = 0
        tseq[:Bp] = np.arange(Bp)
        rows = np.fromiter((s.row for s in launch), dtype=np.int64, count=len(launch))
        p = np.fromiter((s.n_fed for s in launch), dtype=np.int64, count=len(launch))
        up = np.fromiter((id(s) in prev for s in launch), dtype=bool, count=len(launch))
        ids[rows] = [0 if u else s.tokens[-1] for s, u in zip(launch, up)]
        usep[rows] = up
        pos[rows] = p
        ctxl[rows] = p + 1
        slot[rows] = bt[rows, p // self.bs] * self.bs + p % self.bs
        return Bp

    def _launch(self, launch: List[_Seq], prev: set, need: bool = False, dsamp: bool = False):
        if not need:
            self._cand_mode = False
        t0 = time.perf_counter()
        try:
            return self._launch_inner(launch, prev, need, dsamp)
        finally:
            self.host_ms["launch"] += (time.perf_counter() - t0) * 1e3

    def _launch_inner(self, launch: List[_Seq], prev: set, need: bool, dsamp: bool):
        k = self._kbuf = self._kbuf ^ 1
        srows = None
        if self.device_sampling:
            if self.tp is not None and self._srow_dirty:     # followers get the same rows with the step
                srows = [(r,) + v for r, v in sorted(self._srow_dirty.items())]
            self._flush_sampling_rows(k)
        Bp = self._build_meta(k, launch, prev)
        pad = self.db.pad
        self._ctrl(_OP_DECODE, Bp, 0, need, [], Bp, self.h_meta_d2[k], pad, dsamp=dsamp, srows=srows)
        b = self.db
        if self.dev.type == "cuda":
            b.meta.copy_(self.h_meta_d2[k], non_blocking=True)
        else:
            b.meta.copy_(self.h_meta_d2[k])
        self._run_decode(Bp, need, dsamp)
        if dsamp:
            self.counters["device_sampled_steps"] += 1
        for s in launch:
            s.n_fed += 1
        if self.dev.type == "cuda":
            self.h_next2[k][:Bp].copy_(b.next_ids[:Bp], non_blocking=True)
            if self._oneshot is not None:
                self._oneshot.err_fetch(self.h_err2[k])
            self._ev[k].record()
        else:
            self.h_next2[k][:Bp].copy_(b.next_ids[:Bp])
        self.counters["decode_tokens"] += len(launch)
        return ([(s.row, s) for s in launch], k)

    def _check_comm(self, k: int):
        """Raise (failing the step's requests in _loop) when a tensor-parallel all-reduce of step buffer k
        timed out on any rank: its sums -- and so its tokens -- are not trustworthy. Before raising, every
        rank re-initialises its one-shot buffers (_OP_RESET): late granules of the timed-out call must never
        be taken for a later call's data."""
        if self.h_err2 is not None and int(self.h_err2[k].max()):
            if _TP_TRACE:
                import sys
                print(f"[tp r{self.rank}] one-shot error words (sum, add+norm, gather) {self.h_err2[k].tolist()} "
                      f"after op #{getattr(self, '_nops', 0)}", file=sys.stderr, flush=True)
                print(f"[tp r{self.rank}] state {self._oneshot.debug_state()}", file=sys.stderr, flush=True)
                from ..ops import _lib as _oplib
                if _oplib._OP_TIMING:    # NLS_OP_TIMING: launches whose completion lagged the previous one's
                    print(f"[tp r{self.rank}] op gaps {_oplib.op_timing(50.0)}", file=sys.stderr, flush=True)
            words = self.h_err2[k].tolist()
            for h in self.h_err2:
                h.zero_()
            self._ctrl(_OP_RESET, 0, 0, False, [], 0, None, 0)
            self._oneshot.reset()
            if len(words) > 3 and words[3] == 2:
                raise RuntimeError("expert-parallel row exchange: a received row failed its payload checksum")
            raise RuntimeError("tensor-parallel all-reduce timed out waiting for a peer rank")

    def _process(self, infl):
        snap, k = infl
        if self.dev.type == "cuda":
            t0 = time.perf_counter()
            self._ev[k].synchronize()
            self.host_ms["wait"] += (time.perf_counter() - t0) * 1e3
            self._check_comm(k)
        t0 = time.perf_counter()
        toks = self.h_next2[k].numpy()
        for row, s in snap:
            if not s.done:
                self._append(s, int(toks[row]))
        self.host_ms["tokens"] += (time.perf_counter() - t0) * 1e3

    def _drain(self):
        if self._inflight is not None:
            infl, self._inflight = self._inflight, None
            self._process(infl)
            self._release_rows()

    def _ensure_blocks(self, seqs: List[_Seq]) -> List[_Seq]:
        """Give every sequence about to decode the KV block its next position falls in. When the pool
        cannot cover them, finish the in-flight step first (its finished sequences free blocks), then
        preempt the most recently submitted sequences until it can. Returns the sequences still running."""
        if self.reserve_full:
            return seqs
        bs = self.bs

        def needers():
            return [s for s in seqs if not s.done and s.n_fed < self.ctx and s.n_fed // bs >= len(s.blocks)
                    and len(s.tokens) - s.n_prompt < s.max_new]
        need = needers()
        if len(need) > self.alloc.n_free:
            self._drain()
            seqs = [s for s in seqs if not s.done]
            need = needers()
            # priority is arrival order: the most recently submitted sequences give their blocks up first
            victims = sorted((s for s in self.running if not s.done), key=lambda x: x.t_submit)
            while len(need) > self.alloc.n_free and len(victims) > 1:
                v = victims.pop()
                self._preempt(v)
                seqs = [s for s in seqs if s is not v]
                need = [s for s in need if s is not v]
        for s in need:
            b = self.alloc.alloc(1)
            if b is None:                      # cannot happen: one sequence always fits the pool
                raise RuntimeError("KV pool exhausted by a single sequence")
            s.blocks.append(b[0])
            if s.row >= 0:
                for hm in self.h_meta_d2:
                    hm.numpy()[_NSEG * self.db.pad:].reshape(self.max_batch, self.max_blocks)[s.row, len(s.blocks) - 1] = b[0]
        return seqs

    def _preempt(self, s: _Seq):
        """Recompute preemption (no step in flight): free the sequence's blocks and decode row and put it
        back at the head of the queue; it is re-prefilled from prompt + generated tokens (the prefix cache
        usually still holds its prompt blocks) and its stream continues where it stopped."""
        self.alloc.release(s.blocks)
        s.blocks = []
        if s.row >= 0:
            self.rows[s.row] = None
            s.row = -1
        s.n_target = len(s.tokens)
        s.n_prefilled = s.n_cached = 0
        s.n_fed = 0
        s.preempted += 1
        self.counters["preemptions"] += 1
        self._pressure_until = self.counters["steps"] + self.PRESSURE_STEPS
        self.counters["recompute_tokens"] += s.n_target
        self.running = [x for x in self.running if x is not s]
        with self.lock:
            self.waiting.appendleft(s)

    def _decode(self, seqs: List[_Seq]):
        for s in seqs:
            if s.row < 0:
                self._assign_row(s)
        seqs = self._ensure_blocks(seqs)
        if not seqs:
            self._drain()
            return
        greedy = all(s.req.params.greedy for s in seqs)
        # sampled rows drawn inside the decode graph (tensor parallel: when the candidates are exact for
        # every sampled row of the step, else the host-driven full-logits path)
        dsamp = not greedy and self.device_sampling and (self.tp is None or self._cand_ok(seqs))
        chain = self.async_decode and (greedy or dsamp)
        if not chain:
            self._drain()
        n_rows = max(s.row for s in seqs) + 1
        if self._bucket(n_rows) > self._bucket(len(seqs)) and self._inflight is None:
            self._compact(seqs)
        infl = self._inflight
        prev = set(id(s) for _, s in infl[0]) if infl is not None else set()
        launch = []
        for s in seqs:
            ahead = 1 if id(s) in prev else 0
            if len(s.tokens) - s.n_prompt + ahead >= s.max_new or s.n_fed >= self.ctx:
                continue                       # finishes (length) with the step in flight
            launch.append(s)
        if not chain:
            # synchronous step (sampling / penalties need the host between steps)
            need = any(not s.req.params.greedy for s in launch)
            self._cand_mode = need and self._cand_ok(launch)
            new = self._launch(launch, prev, need) if launch else None
            if new is not None:
                self._process_sync(new, launch, need)
            self._release_rows()
            return
        new = self._launch(launch, prev, dsamp=dsamp) if launch else None
        self._inflight = None
        if infl is not None:
            self._process(infl)
        self._inflight = new
        self._release_rows(keep=[s for _, s in new[0]] if new is not None else ())

    def _process_sync(self, new, launch: List[_Seq], need: bool):
        snap, k = new
        b = self.db
        rows = [r for r, _ in snap]
        if self.dev.type == "cuda":
            self._ev[k].synchronize()
            self._check_comm(k)
        greedy = self.h_next2[k].numpy()
        out = [int(greedy[r]) for r in rows]
        sampled = [i for i, s in enumerate(launch) if not s.req.params.greedy]
        if need:                               # (TP: followers gather in the same step)
            self._gather(b, self._bucket(max(rows) + 1), True)
        if sampled and self.cand is not None:
            toks = self._sample_candidates([rows[i] for i in sampled], [launch[i] for i in sampled])
            for i, t in zip(sampled, toks):
                out[i] = t
            sampled = []
        if sampled:
            lg = self.full_logits if self.full_logits is not None else b.logits
            fn = sample_rows_gpu if lg.is_cuda else sample_rows
            toks = fn(lg[[rows[i] for i in sampled]], [launch[i].req.params for i in sampled],
                      [launch[i].tokens for i in sampled], [self._u(launch[i]) for i in sampled])
            for i, t in zip(sampled, toks):
                out[i] = t
        for s, t in zip(launch, out):
            if not s.done:
                self._append(s, t)
        if self.device_sampling:
            # host-drawn tokens never reach the device penalty-history ring (the in-step sampler appends only
            # its own draws): re-stage every sampling row still running, so a later in-step draw penalises
            # the right tokens (the staged rows ship to followers with the next step)
            for s in launch:
                if not s.done and s.row >= 0 and not s.req.params.greedy:
                    self._upload_sampling_row(s.row, s)

    def _step_forward(self, Bp: int, ns: int, need_logits: bool, dsamp: bool):
        self.model.forward(self.db, self.kc, self.vc, Bp, self.bs, ns, feed_prev=True,
                           need_logits=need_logits or dsamp)
        if dsamp:
            b = self.db
            if self.tp is None:
                ops.sample_decode(b.logits, Bp, self.d_sparams, self.d_seeds, b.pos, b.ctx_len, self.d_hist,
                                  b.next_ids)
                return
            m = self.model
            valid = max(0, min(m.vocab_hi, m.cfg.vocab) - m.vocab_lo)
            cv, ci = self.tp.gather_candidates(*ops.topc_candidates(b.logits, Bp, self.CAND, m.vocab_lo, valid))
            ops.sample_decode_cand(cv.contiguous(), ci.contiguous(), Bp, self.d_sparams, self.d_seeds, b.pos,
                                   b.ctx_len, self.d_hist, b.next_ids)

    def _run_decode(self, Bp: int, need_logits: bool = False, dsamp: bool = False):
        ns = LlamaModel.attn_splits(Bp, self.model.Hkv)
        if not self.use_graphs:
            self._step_forward(Bp, ns, need_logits, dsamp)
            return
        key = (Bp, need_logits, dsamp) if dsamp else (Bp, need_logits)
        g = self.graphs.get(key)
        if g is None:
            # first use of this graph (TP followers, sampled / logits variants): THIS step runs eagerly --
            # exactly once, it has side effects (chained ids, KV append, history ring) -- and the capture
            # that follows only records the kernels for the next steps
            self._step_forward(Bp, ns, need_logits, dsamp)
            self._capture(Bp, ns, need_logits, dsamp, warm=False)
            return
        if _NO_REPLAY:                          # (diagnostics: graphs captured, every step eager)
            self._step_forward(Bp, ns, need_logits, dsamp)
            return
        g.replay()
        self.counters["graph_replays"] += 1

    def _capture(self, Bp: int, ns: int, need_logits: bool = False, dsamp: bool = False, warm: bool = True):
        # eager warm-up allocates every lazily sized workspace before capture (callers whose step already
        # ran eagerly pass warm=False)
        if warm:
            self._step_forward(Bp, ns, need_logits, dsamp)
        torch.cuda.synchronize(self.dev)
        dump = os.environ.get("NLS_GRAPH_DUMP")
        g = torch.cuda.CUDAGraph(keep_graph=True) if dump else torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step_forward(Bp, ns, need_logits, dsamp)
        torch.cuda.synchronize(self.dev)
        if dump:
            # (diagnostics) the captured graph's kernel nodes by name, one file per graph: proves e.g. that a TP
            # decode graph holds no RCCL call (parallel/rehearsal.py summarises the dumps)
            import ctypes
            os.makedirs(dump, exist_ok=True)
            buf = ctypes.create_string_buffer(1 << 20)
            n = ops._lib.lib().nls_graph_kernel_names(g.raw_cuda_graph(), buf, len(buf))
            with open(os.path.join(dump, f"w{self.model.shard.size}_r{self.rank}_B{Bp}_logits{int(need_logits)}_dsamp{int(dsamp)}.nodes"),
                      "w") as f:
                f.write(f"# {n} nodes\n" + buf.value.decode(errors="replace"))
            g.instantiate()
        self.graphs[(Bp, need_logits, dsamp) if dsamp else (Bp, need_logits)] = g
        return g

    def _precapture_prefill(self):
        """Capture every single-prompt prefill graph on dummy metadata: every row slot -1 (no KV writes), one query
        block over the whole bucket at position 0 of sequence 0 (its reads land in valid blocks, the outputs are
        discarded)."""
        if not (self.use_graphs and _PREFILL_GRAPHS and self.tp is None and self.model.cfg.n_expert == 0
                and self.prefill_attn):
            return
        self._pf_buffers()
        b, pad = self.pb, self.pb.pad
        h = self.h_meta_p.numpy()
        ld, qd = self._pf_dev
        for Tb in self.PREFILL_GRAPH_T:
            if Tb > self.max_prefill:
                continue
            h[:_NSEG * pad] = 0
            h[2 * pad:3 * pad] = -1
            h[_NSEG * pad:] = 0
            b.meta.copy_(self.h_meta_p)
            ld.zero_()
            qd[0] = torch.tensor([0, Tb, 0, 0], dtype=torch.int32)
            for need in (False, True):
                if (Tb, need) not in self.pf_graphs:
                    self._pf_forward(Tb, need)
                    self._capture_prefill((Tb, need))
        torch.cuda.synchronize(self.dev)

    def capture_all(self, buckets: Seq[int] = None):
        """Pre-capture decode graphs (padded rows have ctx 0 / slot -1: no KV writes) and the single-prompt
        prefill graphs."""
        if not self.use_graphs:
            return
        self._drain()
        self._precapture_prefill()
        pad = self.db.pad
        h = self.h_meta_d2[0].numpy()
        h[:_NSEG * pad] = 0
        h[2 * pad:3 * pad] = -1
        self.db.meta.copy_(self.h_meta_d2[0])
        for Bp in buckets or [k for k in BUCKETS if k <= self.max_batch]:
            if (Bp, False) not in self.graphs:
                self._ctrl(_OP_CAPTURE, Bp, 0, False, [], 0, None, 0)
                self._capture(Bp, LlamaModel.attn_splits(Bp, self.model.Hkv))
            # the in-graph sampling variant too (on every rank): captured lazily, it stalls the first sampled
            # burst at every bucket (an eager step + capture + two device syncs each, ~0.2-0.4 s over a
            # 512-request ramp). Padded rows have ctx 0 and every row's params are greedy here: no history writes.
            if self.device_sampling and (Bp, False, True) not in self.graphs:
                self._ctrl(_OP_CAPTURE, Bp, 0, False, [], 0, None, 0, dsamp=True)
                self._capture(Bp, LlamaModel.attn_splits(Bp, self.model.Hkv), dsamp=True)

    # ------------------------------------------------------------------ completion
    def _append(self, s: _Seq, t: int):
        s.tokens.append(int(t))
        p = s.req.params
        if s.req.on_token is not None:
            try:
                s.req.on_token(int(t))
            except Exception:
                pass
        ng = len(s.tokens) - s.n_prompt
        if not p.ignore_eos and int(t) in self.eos:
            self._finish(s, "stop", "eosFound")
        elif int(t) in p.stop_token_ids:
            self._finish(s, "stop", "stopTokenFound")
        elif p.stop and self.tok is not None and self._stop_string(s):
            self._finish(s, "stop", "stopStringFound")
        elif ng >= s.max_new:
            self._finish(s, "length", "maxPredictedTokensReached")
        elif len(s.tokens) >= self.ctx:
            self._finish(s, "length", "contextLengthReached")

    def _stop_string(self, s: _Seq) -> bool:
        """Incremental: the generated text grows by the stream decoder's delta and only its tail that a
        new occurrence could overlap is searched (decoding the whole generation every step is O(n^2)
        host work per request, paid on the engine thread)."""
        if s.text_cache is None:
            from ..tokenizer.bpe import StreamDecoder
            sd = StreamDecoder(self.tok)
            for t in s.generated[:-1]:
                sd.push(t)
            s.text_cache = [sd, ""]
        sd, text = s.text_cache
        delta = sd.push(s.tokens[-1])
        if not delta:
            return False
        text += delta
        s.text_cache[1] = text
        for st in s.req.params.stop:
            if st and st in text[-(len(st) + len(delta)):]:
                return True
        return False

    def _finish(self, s: _Seq, finish: str, reason: str, error: str = None):
        if s.done:
            return
        s.done = True
        s.t_done = time.monotonic()
        if finish in ("stop", "length") and s.max_new > 0:     # admission's expected-growth estimate
            self.gen_ratio += 0.1 * (min(1.0, (len(s.tokens) - s.n_prompt) / s.max_new) - self.gen_ratio)
        if s.blocks:
            self.alloc.release(s.blocks)
            s.blocks = []
        gen = s.generated
        text = ""
        if self.tok is not None:
            text = self.tok.decode(gen)
            if reason == "stopStringFound":
                cut = min((text.find(st) for st in s.req.params.stop if st and st in text), default=-1)
                if cut >= 0:
                    text = text[:cut]
        gen_ids = gen
        t_first = s.t_first or s.t_done
        res = GenResult(s.req.request_id, gen_ids, text, s.n_prompt, len(gen), finish, reason,
                        t_first - s.t_submit, max(s.t_done - t_first, 1e-9), error,
                        s.t_submit, s.t_admit or s.t_done, t_first, s.t_done)
        if not s.fut.done():
            s.fut.set_result(res)

    def stats(self) -> dict:
        return dict(self.counters, running=len(self.running), waiting=len(self.waiting),
                    kv_blocks_free=self.alloc.n_free, kv_blocks_total=self.num_blocks,
                    kv_reserve="full" if self.reserve_full else "ondemand", gen_ratio=round(self.gen_ratio, 3),
                    prefix_cache_hit_tokens=self.alloc.hits, prefix_cache_blocks=len(self.alloc.block_of),
                    graphs=sorted(self.graphs), prefill_graphs=sorted(self.pf_graphs),
                    dense_weight_gb=round(self.dense_bytes / 1e9, 2), dense_policy=self.dense_policy,
                    kv_pool_gb=round(self.kv_pool_bytes / 1e9, 2),
                    host_ms={k: round(v, 1) for k, v in self.host_ms.items()})
