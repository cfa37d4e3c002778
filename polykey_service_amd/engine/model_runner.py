"""Model runner: step inputs → device, forward, logits, sampling; HIP graphs for decode.

Per step the CPU work is one native call (``BlockManager.pack_step`` writes token ids,
positions, slot mapping, block tables, context lengths and query offsets into a pinned
int32 staging buffer), one H2D copy of that buffer, the forward, and one D2H copy of the
sampled ids.  The device-side copy of the staging buffer has fixed section offsets, so its
views are stable and a decode step can be *captured once per batch-size bucket* and replayed
with ``hipGraphLaunch`` (torch.cuda.CUDAGraph on ROCm) — the launch-bound decode loop of
32–80 layers × ~10 kernels collapses into one graph launch (guide: "capture launch-bound
inner loops in hipGraphs").

Tensor parallelism: the TP leader schedules; every other rank of its group runs
:meth:`ModelRunner.worker_loop`.  The leader publishes each step's packed staging bytes (header
included) through a shared-memory ring (``_pk_runtime.StepChannel``, csrc/runtime/step_channel.h);
a worker copies them into its own pinned staging buffer, reads the header on the host and
launches the same graph / kernels at once — no collective and no GPU sync per step on the
control plane.  Decode continuations replicate on workers too: every rank samples the same ids
from the all-gathered logits, so a worker feeds its own previous sampled ids forward.

KV cache: one allocation per layer pair, K ``[blocks, n_kv, bs, 128]`` and transposed V
``[blocks, n_kv, 128, bs]`` (see ops/attention.py), sized from free HBM after weights and
a measured activation peak — at 288 GB per MI355X an 8B model gets ~1.9 M cached tokens.
"""
from __future__ import annotations

import dataclasses
import math
import os
import threading
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ops import attention as attn_ops
from ..ops import gemm
from ..ops import native
from ..ops import sampler as sampler_ops
from .scheduler import ScheduledBatch
from .sequence import Sequence


@dataclasses.dataclass
class RunnerConfig:
    block_size: int = 32
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: int = 8192
    num_kv_blocks: int = 0           # 0 → size from free memory
    gpu_mem_fraction: float = 0.90
    hip_graphs: bool = True
    graph_batch_sizes: Tuple[int, ...] = ()


# Long-context decode merges its partitions in a second kernel (an in-kernel last-arriver merge
# needs an agent-scope release per partition and measured 1.7-1.9x slower at 1-4K contexts,
# tools/bench_attn.py).  Step inputs are staged by a kernel reading pinned memory instead of an
# SDMA copy.  Each decode bucket has a second graph for steps whose contexts all fit one attention
# partition (one workgroup per (seq, kv head), no merge kernel).


class _Layout:
    """Fixed offsets of every per-step int32 section inside one staging buffer."""

    def __init__(self, max_tokens: int, max_seqs: int, max_blocks: int):
        self.max_tokens, self.max_seqs, self.max_blocks = max_tokens, max_seqs, max_blocks
        off = 0
        self.sections = {}
        for name, n in (("header", 16), ("input_ids", max_tokens), ("positions", max_tokens), ("slots", max_tokens),
                        ("context_lens", max_seqs), ("cu_q", max_seqs + 1), ("cu_rel", max_seqs + 1), ("sample_idx", max_seqs),
                        ("temperature", max_seqs), ("top_k", max_seqs), ("top_p", max_seqs), ("min_p", max_seqs),
                        ("seeds", max_seqs), ("offsets", max_seqs), ("block_tables", max_seqs * max_blocks)):
            self.sections[name] = (off, n)
            off += (n + 15) // 16 * 16  # 64-byte aligned sections
        self.size = off

    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        off, n = self.sections[name]
        v = buf[off:off + n]
        if name in ("temperature", "top_p", "min_p"):
            v = v.view(torch.float32)
        if name == "block_tables":
            v = v.view(self.max_seqs, self.max_blocks)
        return v


class TPPeerError(RuntimeError):
    """A rank of this TP group died or stopped responding: the group cannot continue."""


def peer_timeout_ms() -> int:
    """Bound of every wait on a TP peer (step ring slot, IPC collective): POLYKEY_CUSTOM_AR_TIMEOUT_S."""
    return int(float(os.environ.get("POLYKEY_CUSTOM_AR_TIMEOUT_S", "30")) * 1000)


class ModelRunner:
    def __init__(self, model, cfg: RunnerConfig, device: torch.device, block_manager=None):
        self.model = model
        self.bm = block_manager
        self.mcfg = model.cfg
        self.cfg = cfg
        self.device = device
        self.bs = cfg.block_size
        self.max_blocks = (cfg.max_model_len + self.bs - 1) // self.bs
        self.max_step_tokens = cfg.max_num_batched_tokens  # decodes count toward the budget
        self.layout = _Layout(self.max_step_tokens, cfg.max_num_seqs, self.max_blocks)
        pin = device.type == "cuda"
        # two pinned staging buffers used alternately: a step may be packed while the previous
        # step's H2D copy is still queued behind the GPU (continuation launches, LLMEngine.step)
        self._host_bufs = [torch.zeros(self.layout.size, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self._hs = [{k: self.layout.view(b, k).numpy() for k in self.layout.sections} for b in self._host_bufs]
        self._hnp = [b.numpy() for b in self._host_bufs]  # whole-buffer views (step channel I/O)
        self._h2d_events = [None, None]
        self._cur = 0
        self.host_buf, self.h = self._host_bufs[0], self._hs[0]
        self.dev_buf = torch.zeros(self.layout.size, dtype=torch.int32, device=device)
        self.d = {k: self.layout.view(self.dev_buf, k) for k in self.layout.sections}
        self._tok_hosts = [torch.zeros(cfg.max_num_seqs, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self._tok_events = [None, None]
        self._tok_i = 0
        self.kv_caches: List[Tuple[torch.Tensor, torch.Tensor]] = []
        self.num_blocks = 0
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.graph_out: Dict[int, torch.Tensor] = {}
        self.short_graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.short_graph_out: Dict[int, torch.Tensor] = {}
        self.short_ctx = attn_ops._PART if cfg.max_model_len > attn_ops._PART else 0
        self.graph_pool = None
        a0 = model.layers[0].attn
        self.part_o, self.part_ml = attn_ops.decode_workspace(cfg.max_num_seqs, a0.nq, self.max_blocks, self.bs, device,
                                                              kv_heads=a0.nkv)
        self.stats = {"steps": 0, "graph_steps": 0, "short_graph_steps": 0, "tokens": 0}
        self.keep_logits = False  # tests: keep the last eager step's logits
        self.last_logits = None
        # diagnostics (tools/tp_rehearsal.py): every step's logits, graphed steps included (a copy
        # captured into each graph); read last_logits right after the step, before the next one
        self.debug_logits = os.environ.get("POLYKEY_DEBUG_LOGITS") == "1"
        self._graph_logits: Dict[Tuple[int, int], torch.Tensor] = {}
        self.channel = None
        self._prev_toks = None  # worker: last step's sampled ids (device), for continuations
        self.allow_graphs = True  # DP attention + EP: False for steps whose expert all-to-all is not IPC
        if model.st.tp_size > 1:
            self._open_channel()

    # ------------------------------------------------------------- TP control plane
    def _open_channel(self) -> None:
        """Leader creates the step ring in /dev/shm and tells its group the name (one gloo
        broadcast at start-up); workers attach as consumers tp_rank - 1."""
        import uuid

        from .._native.loader import load_extension
        from ..parallel import comm
        st = self.model.st
        rt = load_extension("_pk_runtime")
        slot_bytes = self.layout.size * 4
        if st.tp_rank == 0:
            name = f"/pk_step_{os.getpid()}_{st.dp_rank}_{uuid.uuid4().hex[:8]}"
            self.channel = rt.StepChannel(name, True, 4, st.tp_size - 1, slot_bytes)
            comm.tp_broadcast_object(name)
        else:
            name = comm.tp_broadcast_object(None)
            self.channel = rt.StepChannel(name, False, consumer_index=st.tp_rank - 1)
        comm.barrier(st.tp_cpu_group)  # every consumer attached before the first publish
        if st.tp_rank == 0:
            self.channel.unlink()  # nothing left in /dev/shm if the group is killed

    # ---------------------------------------------------------------- KV cache
    def kv_bytes_per_block(self) -> int:
        a = self.model.layers[0].attn
        return 2 * len(self.model.layers) * a.nkv * self.bs * a.hd * 2

    def allocate_kv_cache(self, num_blocks: int = 0) -> int:
        a = self.model.layers[0].attn
        if num_blocks <= 0:
            num_blocks = self.cfg.num_kv_blocks
        if num_blocks <= 0:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
                free, total = torch.cuda.mem_get_info(self.device)
                reserve = self.activation_reserve_bytes()
                usable = free - (1.0 - self.cfg.gpu_mem_fraction) * total - reserve
                num_blocks = int(max(usable, 0) // self.kv_bytes_per_block())
                cap = self.cfg.max_num_seqs * self.max_blocks + 16
                num_blocks = max(16, min(num_blocks, cap))
            else:
                num_blocks = max(16, min(self.cfg.max_num_seqs * self.max_blocks, 4096))
        self.num_blocks = num_blocks
        self.kv_caches = []
        for _ in self.model.layers:
            k = torch.zeros((num_blocks, a.nkv, self.bs, a.hd), dtype=self.model.dtype, device=self.device)
            v = torch.zeros((num_blocks, a.nkv, a.hd, self.bs), dtype=self.model.dtype, device=self.device)
            self.kv_caches.append((k, v))
        return num_blocks

    def activation_reserve_bytes(self) -> int:
        m = self.mcfg
        T = self.max_step_tokens
        tp = self.model.st.tp_size
        per_tok = 2 * (m.hidden_size * 4 + (m.q_size + 2 * m.kv_size) // tp + 3 * m.intermediate_size // tp)
        logits = self.cfg.max_num_seqs * m.vocab_size * 4 * 2
        return int(T * per_tok * 1.5 + logits + (1 << 30))

    # ------------------------------------------------------------------ inputs
    def _pack(self, batch: ScheduledBatch, sampling: List[Sequence]):
        decodes, prefills = batch.decodes, batch.prefills
        seqs = decodes + [s for s, _ in prefills]
        n = len(seqs)
        nnew = np.empty(n, dtype=np.int32)
        ncomp = np.empty(n, dtype=np.int32)
        sids = np.empty(n, dtype=np.int64)
        toks: List[int] = []
        for i, s in enumerate(decodes):
            sids[i], ncomp[i], nnew[i] = s.seq_id, s.num_computed, 1
            toks.append(s.output_ids[-1] if s.output_ids else s.prompt_ids[-1])
        for j, (s, c) in enumerate(prefills):
            i = len(decodes) + j
            sids[i], ncomp[i], nnew[i] = s.seq_id, s.num_computed, c
            toks.extend(s.token_slice(s.num_computed, s.num_computed + c))
        tok_arr = np.asarray(toks, dtype=np.int32)
        h = self.h
        T = self.bm.pack_step(sids, ncomp, nnew, tok_arr, h["input_ids"], h["positions"], h["slots"],
                              h["block_tables"], self.max_blocks, h["context_lens"], h["cu_q"])
        # sampling rows: hidden-state row index of each sampling sequence
        pos_of = {s.seq_id: int(h["cu_q"][i + 1]) - 1 for i, s in enumerate(seqs)}
        for r, s in enumerate(sampling):
            p = s.params
            h["sample_idx"][r] = pos_of[s.seq_id]
            h["temperature"][r] = p.temperature
            h["top_k"][r] = p.top_k
            h["top_p"][r] = p.top_p
            h["min_p"][r] = p.min_p
            h["seeds"][r] = s.seed
            h["offsets"][r] = len(s.output_ids)
        return T, n

    def _metadata(self, nd: int, n: int, T: int, max_q: int, short: bool = False) -> attn_ops.AttnMetadata:
        """``short``: every decode context is at most ``self.short_ctx`` tokens."""
        d = self.d
        npf = n - nd
        md = attn_ops.AttnMetadata(
            num_decode=nd, num_prefill=npf, num_prefill_tokens=T - nd, max_prefill_q_len=max_q,
            slot_mapping=d["slots"][:T],
            decode_block_tables=d["block_tables"][:nd] if nd else None,
            decode_context_lens=d["context_lens"][:nd] if nd else None,
            decode_part_o=self.part_o, decode_part_ml=self.part_ml,
            decode_max_ctx=self.short_ctx if short else 0)
        if npf:
            md.prefill_block_tables = d["block_tables"][nd:n]
            md.prefill_context_lens = d["context_lens"][nd:n]
            # query offsets relative to the first prefill token
            md.prefill_cu_q = d["cu_rel"][:npf + 1]
        return md

    # ----------------------------------------------------------------- execute
    # header words (section "header"): mode, T, n, nd, ns, max_q, graph bucket, short-context graph,
    # continuation (input ids = the previous step's sampled ids, already on the device)
    MODE_IDLE, MODE_RUN, MODE_STOP = 0, 1, 2

    @torch.inference_mode()
    def execute(self, batch: ScheduledBatch) -> List[int]:
        """TP leader / single rank: pack, publish, run.  Returns the sampled token ids of
        ``batch.sampling_seqs()`` in order."""
        return self.fetch(self.launch(batch))

    def _next_staging(self) -> None:
        self._cur ^= 1
        ev = self._h2d_events[self._cur]
        if ev is not None:
            ev.synchronize()  # that buffer's last H2D copy has been consumed (normally long ago)
        self.host_buf, self.h = self._host_bufs[self._cur], self._hs[self._cur]

    def launch(self, batch: ScheduledBatch):
        """Enqueue one step (pack → H2D → graph replay / eager forward → sample → async D2H of
        the sampled ids) without waiting for the GPU; :meth:`fetch` returns the ids."""
        self._next_staging()
        sampling = batch.sampling_seqs()
        T, n = self._pack(batch, sampling)
        nd = len(batch.decodes)
        ns = len(sampling)
        h = self.h
        max_q = 0
        g = 0
        if batch.prefills:
            rel = h["cu_q"][nd:n + 1] - h["cu_q"][nd]
            h["cu_rel"][:n - nd + 1] = rel
            max_q = int(np.max(np.diff(rel)))
        elif self.graphs and self.allow_graphs:
            st = self.model.st
            # DP attention + EP: every rank replays the bucket of the group's largest token count
            # (the lockstep vote's max): a graph's grouped expert GEMMs tile the rows any expert
            # can receive from the bucket it was captured at, so a rank with fewer sequences than
            # its peers must not replay a smaller one
            g = self._graph_bucket(max(nd, st.ep_step_rows) if st.dp_attention else nd) or 0
            if g:
                self._pad_decode(nd, g)
        short = self._short(g, nd)
        h["header"][:9] = (self.MODE_RUN, T, n, nd, ns, max_q, g, short, 0)
        self._publish(max(n, g))
        toks = self._run(T, n, nd, ns, max_q, g, short)
        return self._handle(toks, ns)

    def _short(self, g: int, nd: int) -> int:
        """1 when every decode context fits one attention partition: the step replays bucket
        ``g``'s short-context graph, or (eager, g = 0) launches the same one-workgroup-per-
        (seq, kv head) decode attention -- so eager and graphed steps compute identical sums."""
        if not (self.short_ctx and nd) or (g and g not in self.short_graphs):
            return 0
        return int(int(self.h["context_lens"][:nd].max()) <= self.short_ctx)

    def _handle(self, toks, ns: int):
        self.stats["steps"] += 1
        if ns == 0 or toks is None:
            return None, 0, None, None
        if not toks.is_cuda:
            return toks, ns, None, None
        self._tok_i ^= 1
        host = self._tok_hosts[self._tok_i]
        host[:ns].copy_(toks[:ns], non_blocking=True)
        ev = self._tok_events[self._tok_i]
        if ev is None:
            ev = self._tok_events[self._tok_i] = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return host, ns, ev, toks

    def fetch(self, handle) -> List[int]:
        toks, ns, ev, _ = handle
        if ev is not None:
            ev.synchronize()
        self._check_comm()
        if ns == 0:
            return []
        return toks[:ns].tolist()

    def _check_comm(self) -> None:
        """Fail loudly once a custom all-reduce of this step (or an earlier one) timed out: the
        step's tokens were computed from incomplete sums (parallel/custom_ar.py)."""
        st = self.model.st
        gemm.check_fused()
        if st.custom_ar is not None:
            st.custom_ar.check()
        for rc in (getattr(st, "rccl_tp", None), getattr(st, "rccl_ep", None)):
            if rc is not None:  # RCCL's asynchronous error word (non-blocking poll)
                rc.check()
        for a2a in (getattr(st, "ep_a2a", None), getattr(st, "ep_a2a_prefill", None)):
            if a2a is not None:
                a2a.check()

    def launch_continuation(self, batch: ScheduledBatch, prev) -> Optional[tuple]:
        """Decode step k+1 of ``batch.decodes`` enqueued while step k (``prev``) may still run:
        every sequence advances one position, and step k's sampled ids — still on the GPU —
        are copied into this step's input ids on the stream, so the host never waits between
        the two steps.  Needs a captured graph bucket; returns None (caller falls back to a
        scheduled step) when a sequence cannot get the KV block for its next position."""
        seqs = batch.decodes
        n = len(seqs)
        g = self._graph_bucket(n) if self.graphs else None
        if not g or prev[3] is None or batch.prefills:
            return None
        for s in seqs:
            if s.num_computed + 2 > self.cfg.max_model_len or not self.bm.allocate(s.seq_id, s.num_computed + 2):
                return None
        self._next_staging()
        h = self.h
        sids = np.fromiter((s.seq_id for s in seqs), dtype=np.int64, count=n)
        ncomp = np.fromiter((s.num_computed + 1 for s in seqs), dtype=np.int32, count=n)
        ones = np.ones(n, dtype=np.int32)
        T = self.bm.pack_step(sids, ncomp, ones, np.zeros(n, dtype=np.int32), h["input_ids"], h["positions"],
                              h["slots"], h["block_tables"], self.max_blocks, h["context_lens"], h["cu_q"])
        h["sample_idx"][:n] = np.arange(n, dtype=np.int32)
        for r, s in enumerate(seqs):
            p = s.params
            h["temperature"][r] = p.temperature
            h["top_k"][r] = p.top_k
            h["top_p"][r] = p.top_p
            h["min_p"][r] = p.min_p
            h["seeds"][r] = s.seed
            h["offsets"][r] = len(s.output_ids) + 1
        self._pad_decode(n, g)
        short = self._short(g, n)
        h["header"][:9] = (self.MODE_RUN, T, n, n, n, 0, g, short, 1)
        self._publish(max(n, g))
        self.d["input_ids"][:n].copy_(prev[3][:n])  # step k's sampled ids, stream-ordered
        return self._handle(self._run(T, n, n, n, 0, g, short), n)

    def _staged_words(self, n_bt_rows: Optional[int]) -> int:
        """int32 words of the staging buffer a step uses: everything up to the used block-table
        rows (the last section), rounded to 16 bytes."""
        off, _ = self.layout.sections["block_tables"]
        rows = self.cfg.max_num_seqs if n_bt_rows is None else n_bt_rows
        n = min(self.layout.size, off + rows * self.max_blocks)
        return (n + 3) // 4 * 4

    def _publish(self, n_bt_rows: Optional[int] = None) -> None:
        """Hand the step inputs to the TP workers (shared-memory ring, host to host) and stage
        them on this rank's device.  The wait for a slot is bounded by the collectives' timeout:
        a worker that died (its pid is gone) or stopped consuming fails the step loudly."""
        n = self._staged_words(n_bt_rows)
        if self.channel is not None and self.model.st.tp_rank == 0:
            if not self.channel.publish(self._hnp[self._cur], n * 4, peer_timeout_ms()):
                dead = self.channel.dead_consumer()
                who = f"TP rank {dead + 1} died" if dead >= 0 else "a TP worker stopped consuming steps"
                raise TPPeerError(f"TP step channel: {who}")
        self._stage_local(n)

    def _stage_local(self, n: int) -> None:
        """Copy the first ``n`` words of the current pinned staging buffer to the device.  On
        the GPU a kernel reads the pinned buffer directly (no SDMA hand-off)."""
        if self.device.type == "cuda":
            native.call("pk_copy_from_host", self.dev_buf.data_ptr(), self.host_buf.data_ptr(), n * 4,
                        native.stream_ptr(self.device))
        else:
            self.dev_buf[:n].copy_(self.host_buf[:n], non_blocking=True)
        if self.device.type == "cuda":
            ev = self._h2d_events[self._cur]
            if ev is None:
                ev = self._h2d_events[self._cur] = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))

    def worker_loop(self) -> None:
        """Non-leader TP ranks: take each step from the leader's ring into the next pinned
        staging buffer, read its header on the host and launch the same work — the worker never
        waits for its own GPU (only, through the double-buffered staging, for a step two back)."""
        chan = self.channel
        done = threading.Event()
        watch = threading.Thread(target=self._leader_watch, args=(done,), name="pk-leader-watch", daemon=True)
        watch.start()
        try:
            self._worker_steps(chan)
        finally:
            done.set()
            watch.join(5.0)

    def _leader_watch(self, done: threading.Event, grace_s: float = 10.0) -> None:
        """A worker blocked on its GPU (a collective waiting for the dead leader, an RCCL kernel
        that never times out) cannot reach the step channel's dead-producer check: this thread
        sees the leader's pid vanish, aborts the communicators (the waits return), and if the
        main loop has not ended the process ``grace_s`` later, exits it non-zero itself."""
        while not done.wait(1.0):
            if self.channel.producer_alive:
                continue
            self.abort_comms()
            if done.wait(grace_s):
                return
            import sys
            print("TP leader process died and this worker is still blocked on the GPU: exiting",
                  file=sys.stderr, flush=True)
            os._exit(1)

    def _worker_steps(self, chan) -> None:
        while True:
            self._next_staging()
            nbytes = chan.consume(self._hnp[self._cur], 1000)
            self._check_comm()
            if nbytes == -1:
                continue  # idle leader: poll again (and re-check the comm error word)
            if nbytes == -2:
                return
            if nbytes == -3:  # the leader's process is gone (SIGKILL, OOM, crash): end this rank
                raise TPPeerError("TP leader process died; this worker exits for its supervisor to restart the group")
            mode, T, n, nd, ns, max_q, g, short, cont = (int(v) for v in self.h["header"][:9])
            if mode == self.MODE_STOP:
                return
            if mode != self.MODE_RUN:
                continue
            self._stage_local(nbytes // 4)
            with torch.inference_mode():
                if cont:
                    self.d["input_ids"][:n].copy_(self._prev_toks[:n])
                toks = self._run(T, n, nd, ns, max_q, g, short)
            if toks is not None:
                self._prev_toks = toks
            self.stats["steps"] += 1

    def fallback_unfused(self) -> None:
        """A fused decode launch lost an in-launch hand-off (another process on this GPU kept part
        of its grid from being resident): wait for the GPU, re-arm the sticky word, switch this
        process to the two-launch path for good (WARN) and re-capture the decode graphs that held
        the fused kernels.  The caller re-runs the step (LLMEngine._complete_or_redo)."""
        import logging
        logging.getLogger(__name__).warning(
            "fused decode launch hand-off timed out (GPU shared with another process?): the failed step is "
            "re-run and every later step takes the two-launch path")
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        gemm.disable_fused()
        gemm.clear_fused_error()
        self.stats["fused_fallbacks"] = self.stats.get("fused_fallbacks", 0) + 1
        if self.graphs:
            sizes = sorted(self.graphs)
            self.graphs.clear()
            self.graph_out.clear()
            self.short_graphs.clear()
            self.short_graph_out.clear()
            self._graph_logits.clear()
            self.graph_pool = None
            self.capture_graphs(sizes)

    def abort_comms(self) -> None:
        """Watchdog / failure path: tear down this rank's RCCL communicators (a collective hung on
        a dead peer returns) and mark the IPC collectives failed (every later call skips its
        waits), so the process can exit instead of blocking in a GPU wait."""
        st = self.model.st
        for rc in {id(c): c for c in (getattr(st, "rccl_tp", None), getattr(st, "rccl_ep", None))
                   if c is not None}.values():
            try:
                rc.abort()
            except Exception:  # noqa: BLE001 - best effort on the way down
                pass
        if st.custom_ar is not None:
            st.custom_ar.fail()
        for a2a in (getattr(st, "ep_a2a", None), getattr(st, "ep_a2a_prefill", None)):
            if a2a is not None:
                a2a.fail()

    def stop_workers(self) -> None:
        if self.channel is not None and self.model.st.tp_rank == 0:
            self._next_staging()
            self.h["header"][:9] = (self.MODE_STOP, 0, 0, 0, 0, 0, 0, 0, 0)
            self.channel.publish(self._hnp[self._cur], 64, 60000)
            self.channel.close()

    def _run(self, T: int, n: int, nd: int, ns: int, max_q: int, g: int, short: int = 0):
        d = self.d
        if g:
            if short:
                self.short_graphs[g].replay()
                self.stats["short_graph_steps"] += 1
                out = self.short_graph_out[g]
            else:
                self.graphs[g].replay()
                out = self.graph_out[g]
            self.stats["graph_steps"] += 1
            if self.debug_logits:
                self.last_logits = self._graph_logits[(g, int(bool(short)))]
            return out
        md = self._metadata(nd, n, T, max_q, bool(short))
        hidden = self.model(d["input_ids"][:T], d["positions"][:T], md, self.kv_caches)
        if ns == 0:
            return None
        rows = hidden if ns == T else hidden.index_select(0, d["sample_idx"][:ns].long())
        logits = self.model.compute_logits(rows)
        if self.keep_logits or self.debug_logits:
            self.last_logits = logits
        return sampler_ops.sample(logits, d["temperature"][:ns], d["top_k"][:ns], d["top_p"][:ns],
                                  d["min_p"][:ns], d["seeds"][:ns], d["offsets"][:ns])

    # ------------------------------------------------------------------ graphs
    def _graph_bucket(self, nd: int) -> Optional[int]:
        for b in sorted(self.graphs):
            if b >= nd:
                return b
        return None

    def _pad_decode(self, nd: int, g: int) -> None:
        h = self.h
        if g > nd:
            h["input_ids"][nd:g] = 0
            h["positions"][nd:g] = 0
            h["slots"][nd:g] = -1
            h["context_lens"][nd:g] = 0
            h["sample_idx"][nd:g] = np.arange(nd, g, dtype=np.int32)
            h["temperature"][nd:g] = 0.0
            h["top_k"][nd:g] = 0
            h["top_p"][nd:g] = 1.0
            h["min_p"][nd:g] = 0.0

    def default_graph_sizes(self) -> List[int]:
        if self.cfg.graph_batch_sizes:
            sizes = list(self.cfg.graph_batch_sizes)
        else:
            sizes = [1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512]
        return [s for s in sizes if s <= self.cfg.max_num_seqs]

    @torch.inference_mode()
    def capture_graphs(self, sizes: Optional[List[int]] = None) -> None:
        if self.device.type != "cuda" or not self.cfg.hip_graphs:
            return
        sizes = sizes or self.default_graph_sizes()
        st = self.model.st
        if st.dp_attention:  # every replay sends bucket x top-k rows per peer: within the IPC capacity
            k = self.mcfg.experts_per_token
            sizes = [g for g in sizes if st.ep_a2a is not None and st.ep_a2a.fits(g * k)]
        d = self.d
        # a valid dummy decode state: every row points at block 0, context 1, no cache writes
        self.host_buf.zero_()
        self.h["slots"][:] = -1
        self.h["context_lens"][: self.cfg.max_num_seqs] = 1
        self.h["top_p"][:] = 1.0
        self.h["sample_idx"][: self.cfg.max_num_seqs] = np.arange(self.cfg.max_num_seqs, dtype=np.int32)
        self.dev_buf.copy_(self.host_buf)
        torch.cuda.synchronize(self.device)
        stream = torch.cuda.Stream(self.device)
        variants = (False, True) if self.short_ctx else (False,)
        st = self.model.st
        for g, short in [(g, v) for g in sorted(sizes, reverse=True) for v in variants]:
            md = self._metadata(g, g, g, 0, short)
            if st.dp_attention:  # capture the IPC expert all-to-all path (device-side counts)
                st.ep_step_rows = g

            def run():
                hidden = self.model(d["input_ids"][:g], d["positions"][:g], md, self.kv_caches)
                logits = self.model.compute_logits(hidden)
                if self.debug_logits:
                    self._graph_logits[(g, int(short))] = logits.clone()
                return sampler_ops.sample(logits, d["temperature"][:g], d["top_k"][:g], d["top_p"][:g],
                                          d["min_p"][:g], d["seeds"][:g], d["offsets"][:g])

            # warm up on a side stream (allocator + library handles), then capture
            stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(stream):
                run()
            torch.cuda.current_stream(self.device).wait_stream(stream)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, pool=self.graph_pool):
                out = run()
            if self.graph_pool is None:
                self.graph_pool = graph.pool()
            (self.short_graphs if short else self.graphs)[g] = graph
            (self.short_graph_out if short else self.graph_out)[g] = out
        torch.cuda.synchronize(self.device)
