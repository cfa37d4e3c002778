"""Synchronous engine: add requests, ``step()`` until done (the L5 engine of SURVEY.md §3.6).

``step()`` = schedule → model runner (pack, H2D, forward / graph replay, sample, D2H) →
append tokens, detect stop conditions, free finished sequences → per-request outputs.
The async/gRPC face is :mod:`polykey_service_amd.engine.async_llm`.
"""
from __future__ import annotations

import dataclasses
import os
import time
import uuid
from typing import Callable, Dict, Iterable, List, Optional

import torch

from .._native.loader import load_extension
from ..models import build_model
from ..models.config import ModelConfig, get_config
from ..parallel.state import ParallelState, get_state
from .model_runner import ModelRunner, RunnerConfig
from .scheduler import ScheduledBatch, Scheduler
from .sequence import FinishReason, RequestOutput, SamplingParams, Sequence, seq_metrics
from .tokenizer import get_tokenizer


@dataclasses.dataclass
class EngineConfig:
    model: str = "llama3-8b"
    model_path: str = ""
    tokenizer: str = ""
    dtype: str = "bfloat16"
    seed: int = 0
    block_size: int = 32
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: int = 8192
    num_kv_blocks: int = 0
    gpu_mem_fraction: float = 0.90
    hip_graphs: bool = True
    graph_batch_sizes: tuple = ()
    watermark: float = 0.01
    device: str = ""
    overlap: bool = False  # pipelined steps (see LLMEngine.step); AsyncLLM turns it on
    # scheduler policy (engine/scheduler.py): prefill_first | decode_first (decode_first measured
    # slower on the headline wave: profiles/r2_decode_ab.txt "scheduler policy")
    sched_policy: str = "prefill_first"
    max_decode_stall: int = 4
    # > 0: keep only the first num_layers decoder layers of the preset (rehearsals of a large
    # model's per-rank shapes with fewer layers, tests); 0: the preset's depth
    num_layers: int = 0
    # automatic prefix caching (csrc/runtime/block_manager.h); POLYKEY_PREFIX_CACHING=0 disables
    prefix_caching: bool = dataclasses.field(
        default_factory=lambda: os.environ.get("POLYKEY_PREFIX_CACHING", "1") != "0")

    @classmethod
    def from_server_config(cls, sc) -> "EngineConfig":
        return cls(model=sc.model, model_path=sc.model_path, tokenizer=sc.tokenizer, dtype=sc.dtype, seed=sc.seed,
                   block_size=sc.kv_block_size, max_num_seqs=sc.max_num_seqs,
                   max_num_batched_tokens=sc.max_num_batched_tokens, max_model_len=sc.max_model_len,
                   num_kv_blocks=sc.num_kv_blocks, gpu_mem_fraction=sc.gpu_mem_fraction, hip_graphs=sc.hip_graphs,
                   num_layers=getattr(sc, "num_layers", 0))


def tokenizer_for(cfg: EngineConfig, mcfg: Optional[ModelConfig] = None):
    """The tokenizer an engine for ``cfg`` uses (a front end routing to an engine in another
    process builds the same one without the engine)."""
    from .chat_template import family_for
    mcfg = mcfg or get_config(cfg.model_path or cfg.model)
    return get_tokenizer(cfg.tokenizer, mcfg.vocab_size, mcfg.bos_token_id, mcfg.eos_token_id,
                         family_for(mcfg.name, mcfg.is_moe))


class LLMEngine:
    def __init__(self, cfg: EngineConfig, st: Optional[ParallelState] = None, model=None):
        self.cfg = cfg
        self.st = st or get_state()
        mcfg: ModelConfig = get_config(cfg.model_path or cfg.model)
        if cfg.num_layers > 0 and cfg.num_layers != mcfg.num_layers:
            mcfg = dataclasses.replace(mcfg, num_layers=cfg.num_layers)
        if cfg.max_model_len > mcfg.max_position:
            cfg = dataclasses.replace(cfg, max_model_len=mcfg.max_position)
            self.cfg = cfg
        if cfg.block_size <= 0 or cfg.block_size % 32:
            # the K cache stores 32-token fragment-native tiles (csrc/kernels/common.h kcache_off)
            raise ValueError(f"block_size must be a positive multiple of 32, got {cfg.block_size}")
        # DP attention + EP (ParallelState.dp_attention): every rank schedules its own requests
        # and the ranks step in lockstep because each MoE layer is an all-to-all over all of
        # them.  Steps are synchronous (no overlap / continuations).  With the IPC expert
        # all-to-all (parallel/ep_ipc.py: device-side counts) decode steps replay HIP graphs;
        # without it (multi-node, CPU) the dispatch sizes are read back per layer: eager only.
        self.lockstep = self.st.dp_attention
        if self.lockstep:
            if not mcfg.is_moe:
                raise ValueError("DP attention + EP (tp=1, ep>1) needs an MoE model")
            from ..parallel import ep_ipc
            if self.st.ep_a2a is None:
                self.st.ep_a2a = ep_ipc.maybe_create(self.st, cfg.max_num_seqs * mcfg.experts_per_token,
                                                     mcfg.hidden_size)
            if self.st.ep_a2a is not None and self.st.ep_a2a_prefill is None:
                # prefill-sized steps: a second set of regions sized for the token budget (eager,
                # host-free counts too: no per-layer read-back of the split sizes)
                self.st.ep_a2a_prefill = ep_ipc.maybe_create(
                    self.st, max(cfg.max_num_batched_tokens, cfg.max_num_seqs) * mcfg.experts_per_token,
                    mcfg.hidden_size)
            if self.st.ep_a2a is not None and os.environ.get("POLYKEY_PREFLIGHT", "1") != "0":
                from ..parallel import preflight  # dispatch / return checked once; a failure -> RCCL path
                preflight.run(self.st, paths=("ep_ipc",))
            cfg = dataclasses.replace(cfg, overlap=False,
                                      hip_graphs=cfg.hip_graphs and self.st.ep_a2a is not None)
            self.cfg = cfg
        self.mcfg = mcfg
        dev = torch.device(cfg.device) if cfg.device else self.st.device
        self.device = dev
        dtype = getattr(torch, cfg.dtype)
        if model is None:
            model = build_model(mcfg, self.st, dtype, dev)
            if cfg.model_path:
                model.load_hf(cfg.model_path)
            else:
                model.init_random(cfg.seed)
        self.model = model
        if hasattr(model, "pack_decode_weights"):
            model.pack_decode_weights()
        self.tokenizer = tokenizer_for(cfg, mcfg)
        rcfg = RunnerConfig(block_size=cfg.block_size, max_num_seqs=cfg.max_num_seqs,
                            max_num_batched_tokens=cfg.max_num_batched_tokens, max_model_len=cfg.max_model_len,
                            num_kv_blocks=cfg.num_kv_blocks, gpu_mem_fraction=cfg.gpu_mem_fraction,
                            hip_graphs=cfg.hip_graphs, graph_batch_sizes=tuple(cfg.graph_batch_sizes))
        self.runner = ModelRunner(model, rcfg, dev)
        self._serving_preflight(mcfg)
        nblocks = self.runner.allocate_kv_cache()
        rt = load_extension("_pk_runtime")
        self.bm = rt.BlockManager(nblocks, cfg.block_size, int(nblocks * cfg.watermark), cfg.prefix_caching)
        self.runner.bm = self.bm
        self.scheduler = Scheduler(self.bm, cfg.max_num_seqs, cfg.max_num_batched_tokens, cfg.max_model_len,
                                   policy=cfg.sched_policy, max_decode_stall=cfg.max_decode_stall)
        if cfg.hip_graphs and dev.type == "cuda":
            self.runner.capture_graphs()
        self.step_count = 0
        self.total_output_tokens = 0
        self.overlap = cfg.overlap
        self._inflight = None
        # called between completing a step and scheduling the next (AsyncLLM: admit the requests
        # that arrived meanwhile)
        self.before_schedule: Optional[Callable[[], None]] = None
        self.continuation_steps = 0

    def _serving_preflight(self, mcfg: ModelConfig) -> None:
        """TP: the fused decode collective checked at the shape serving will replay it at (the
        largest decode graph bucket x hidden, 16 back-to-back calls, graph-replayed) before any
        graph captures it; a mismatch switches the group to the fenced slot protocol or disables
        the custom collectives on every rank (parallel/preflight.py check_custom_ar_serving)."""
        car = self.st.custom_ar
        if car is None or self.st.tp_size < 2 or os.environ.get("POLYKEY_PREFLIGHT", "1") == "0":
            return
        rows = [g for g in self.runner.default_graph_sizes() if car.supports_reduce_residual(g, mcfg.hidden_size)]
        if rows:
            from ..parallel import preflight
            self.preflight_report = preflight.run(self.st, paths=("custom_ar_serving",),
                                                  serving=(max(rows), mcfg.hidden_size))

    # ------------------------------------------------------------------ API
    @property
    def is_leader(self) -> bool:
        return self.st.tp_rank == 0

    def add_request(self, prompt_ids: List[int], params: SamplingParams, request_id: Optional[str] = None,
                    user=None) -> Sequence:
        params.validate(self.cfg.max_model_len)
        if not prompt_ids:
            raise ValueError("empty prompt")
        if max(prompt_ids) >= self.mcfg.vocab_size or min(prompt_ids) < 0:
            raise ValueError("prompt token id out of range")
        seq = Sequence(request_id or uuid.uuid4().hex, prompt_ids, params, self.mcfg.eos_token_id, user)
        self.scheduler.add(seq)
        return seq

    def abort(self, request_id: str) -> Optional[Sequence]:
        return self.scheduler.abort(request_id)

    def has_unfinished(self) -> bool:
        return self.scheduler.has_work() or self._inflight is not None

    def idle_with_waiting(self) -> bool:
        sch = self.scheduler
        return (not sch.running and self._inflight is None and bool(sch.waiting)
                and len(sch.waiting) < sch.max_num_seqs)

    def first_step_unfilled(self) -> bool:
        """Idle engine (nothing running or in flight) whose waiting requests do not yet fill one
        prefill step (token budget and sequence cap): a burst of arrivals may still be landing."""
        sch = self.scheduler
        if sch.running or self._inflight is not None or not sch.waiting:
            return False
        if len(sch.waiting) >= sch.max_num_seqs:
            return False
        return sum(s.num_pending for s in sch.waiting) < sch.max_num_batched_tokens

    def step(self) -> List[RequestOutput]:
        """One engine iteration.  With ``overlap`` the step is pipelined: the batch launched by
        the previous call is completed (wait for its sampled ids, advance sequence state, free
        finished sequences), the next batch is scheduled and launched, and only then are the
        completed batch's :class:`RequestOutput` objects built and returned — so output
        construction and the caller's delivery of them run while the GPU executes the next
        step.  Without ``overlap`` each call launches and completes its own batch."""
        if self.lockstep:
            return self._step_lockstep()
        done = None
        if self._inflight is not None:
            batch, sampling, handle = self._inflight
            nxt = self._continuation(batch, handle)
            done, redone = self._complete_or_redo(batch, sampling, handle)
            self._inflight = None
            if nxt is not None and not redone:  # a redone step's continuation ran on its bad tokens
                self._inflight = (batch, batch.decodes, nxt)
                self.continuation_steps += 1
                return self._outputs(done)
        if self.before_schedule is not None and done is not None:
            # requests that landed while the completed step ran join the next one (a burst whose
            # tail arrived during the first prefill step is prefilled in the second instead of a
            # straggler third step that delays the whole cohort by a prefill, profiles/r6_gc.md)
            self.before_schedule()
            # a request aborted by it loses the completed step's output too (as an abort while
            # a step is in flight does)
            done = [d for d in done if d[2] is not None or d[0].finish_reason is not FinishReason.ABORT]
        batch = self.scheduler.schedule()
        if not batch.empty:
            sampling = batch.sampling_seqs()
            self._inflight = (batch, sampling, self.runner.launch(batch))
            if not self.overlap:
                done, _ = self._complete_or_redo(*self._inflight)
                self._inflight = None
        return self._outputs(done) if done else []

    def _complete_or_redo(self, batch, sampling, handle):
        """``_complete`` of a launched step; if a fused decode launch of it lost its in-launch
        hand-off (FusedHandoffError: co-tenant on the GPU), the runner falls back to the
        two-launch path and the step is launched again -- the sequences' state is untouched until
        a step completes and the re-run rewrites the same KV slots.  A TP / lockstep group cannot
        re-run one rank alone, so TP ranks that share a GPU (where a co-tenant can starve a
        hand-off) never take the fused launches (models/llama.py _qkv_attn_fused_ok, the fused
        MLP's shared_device check); on a dedicated GPU a lost hand-off is a fault and stays fatal.
        Returns (done, redone)."""
        from ..ops.gemm import FusedHandoffError
        try:
            return self._complete(batch, sampling, handle), False
        except FusedHandoffError:
            if self.st.tp_size > 1 or self.lockstep:
                raise
            self.runner.fallback_unfused()  # drains the GPU: an in-flight continuation is finished
            return self._complete(batch, sampling, self.runner.launch(batch)), True

    def _step_lockstep(self) -> List[RequestOutput]:
        """DP attention + EP step: one lockstep vote (shared memory on one node) per step decides
        whether the EP group runs a forward and -- from the largest token count -- which expert
        all-to-all every rank uses (IPC slots, graph-capturable, for decode-sized steps; RCCL
        for prefill-sized ones); a rank with nothing scheduled joins through the idle pass."""
        from ..parallel import comm
        batch = self.scheduler.schedule()
        ntok = len(batch.decodes) + sum(n for _, n in batch.prefills)
        busy, _, max_tok = comm.ep_vote(not batch.empty, False, ntok)
        if not busy:
            return []
        # (graph buckets pad decode rows, but only buckets within the IPC capacity are captured)
        a2a = self.st.ep_a2a
        ipc = a2a is not None and a2a.fits(max_tok * self.mcfg.experts_per_token)
        # every rank sees the same max: the same regions (decode-sized, prefill-sized or none) on all
        self.st.ep_step_rows = max_tok
        self.runner.allow_graphs = ipc  # a replay holds the IPC path: only when every rank takes it
        if batch.empty:
            self.model.idle_forward()
            self.runner.stats["idle_steps"] = self.runner.stats.get("idle_steps", 0) + 1
            return []
        done = self._complete(batch, batch.sampling_seqs(), self.runner.launch(batch))
        return self._outputs(done)

    def lockstep_vote(self, stopping: bool):
        """DP attention + EP loop vote → (any rank has work, every rank is stopping)."""
        from ..parallel import comm
        busy, all_stop, _ = comm.ep_vote(self.has_unfinished(), stopping)
        return busy, all_stop

    def any_unfinished(self) -> bool:
        """Whether the engine loop must keep stepping: its own work, or (DP attention + EP) any
        rank's -- a collective vote every rank makes once per loop iteration."""
        local = self.has_unfinished()
        if not self.lockstep:
            return local
        from ..parallel import comm
        return comm.ep_any(local)

    def _continuation(self, batch, handle):
        """Launch the next decode step of ``batch`` before its current step has been read back
        (see ModelRunner.launch_continuation) when nothing else could change the batch: pure
        decode, every running sequence in it and alive, no request waiting for admission."""
        sch = self.scheduler
        if (not self.overlap or batch.prefills or sch.waiting or len(batch.decodes) != len(sch.running)
                or any(s.is_finished() for s in batch.decodes)):
            return None
        if all(len(s.output_ids) + 1 >= s.params.max_tokens for s in batch.decodes):
            return None  # the in-flight step ends every sequence: a continuation would be discarded
        return self.runner.launch_continuation(batch, handle)

    def _complete(self, batch, sampling, handle):
        toks = self.runner.fetch(handle)
        now = time.monotonic()
        for s, n in batch.prefills:
            s.num_computed += n
            self.scheduler.commit_prefix(s)  # the step that wrote these blocks' KV has completed
        for s in batch.decodes:
            s.num_computed += 1
        done = []
        for s, tok in zip(sampling, toks):
            if s.is_finished():  # aborted while its step was in flight
                continue
            reason = s.append_token(tok, now)
            if reason is not None:
                self.scheduler.finish(s, reason)
            done.append((s, tok, reason))
        self.scheduler.remove_finished()
        self.step_count += 1
        self.total_output_tokens += len(toks)
        return done

    @staticmethod
    def _outputs(done) -> List[RequestOutput]:
        return [RequestOutput(s.request_id, [tok], reason is not None, reason.value if reason else None,
                              len(s.prompt_ids), len(s.output_ids), seq_metrics(s) if reason else None)
                for s, tok, reason in done]

    def generate(self, prompts: List[List[int]], params: SamplingParams) -> List[List[int]]:
        seqs = [self.add_request(p, dataclasses.replace(params)) for p in prompts]
        while self.any_unfinished():
            self.step()
        return [s.output_ids for s in seqs]

    def shutdown(self) -> None:
        self.runner.stop_workers()
