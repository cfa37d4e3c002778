"""Continuous-batching scheduler (the L3 "Scheduler" of SURVEY.md §1.2 / §3.6).

Every engine step builds one batch under a prefill-token budget (``max_num_batched_tokens``)
and a sequence cap (``max_num_seqs``):

1. running sequences, oldest first: a decode costs 1 token; a sequence still in a chunked
   prefill takes ``min(pending, budget)`` tokens.  If the KV pool cannot grow a
   running sequence, the *youngest* running sequence is preempted (blocks freed, state reset
   to recompute) and the step retries — the oldest requests keep their latency;
2. waiting sequences in FIFO order, admitted only when their (chunked) prefill fits both the
   budget and the KV pool minus a watermark reserve; the first one that does not fit blocks
   the queue (no overtaking → no starvation).

Policy ``prefill_first`` (default, throughput) runs 2 before 1 while prompts are queued —
a wave of prompts is prefilled in whole budget-sized steps (GEMM rows a multiple of the
budget, no small tail chunk needing an extra un-graphed step) — but never skips the running
decodes for more than ``max_decode_stall`` consecutive steps; ``decode_first`` always runs 1
first (lowest inter-token latency under mixed load).

KV bookkeeping lives in the native :class:`_pk_runtime.BlockManager` (``csrc/runtime``).

Automatic prefix caching (block manager built with ``prefix_caching=True``): a sequence
admitted with nothing computed first takes the cached blocks matching the longest prefix of
its tokens (chained block hashes) and starts its prefill after them — leaving at least two
tokens to compute, so it still runs a prefill that samples.  The engine registers a prefill's
full blocks (:meth:`Scheduler.commit_prefix`) once the step that wrote their KV completed.
"""
from __future__ import annotations

import bisect
import collections
import dataclasses
import time
from typing import Deque, Dict, List, Optional, Tuple

import numpy as np

from .sequence import FinishReason, Sequence, SeqStatus


@dataclasses.dataclass
class ScheduledBatch:
    decodes: List[Sequence]
    prefills: List[Tuple[Sequence, int]]   # (seq, chunk length)
    preempted: List[Sequence]

    @property
    def num_tokens(self) -> int:
        return len(self.decodes) + self.num_prefill_tokens

    @property
    def num_prefill_tokens(self) -> int:
        return sum(n for _, n in self.prefills)

    @property
    def empty(self) -> bool:
        return not self.decodes and not self.prefills

    def sampling_seqs(self) -> List[Sequence]:
        """Sequences that produce a token this step (decodes + prefills that finish their prompt)."""
        out = list(self.decodes)
        out += [s for s, n in self.prefills if s.num_computed + n == s.num_tokens]
        return out


def _salt(s: Optional[str]) -> int:
    """Per-request prefix-cache salt (a tenant id): requests only share cached blocks with
    requests of the same salt.  0 = the shared namespace."""
    if not s:
        return 0
    import hashlib
    return int.from_bytes(hashlib.blake2b(s.encode(), digest_size=8).digest(), "little") or 1


class _Step:
    """One step's batch under construction."""

    def __init__(self, budget: int):
        self.budget = budget
        self.decodes: List[Sequence] = []
        self.prefills: List[Tuple[Sequence, int]] = []
        self.preempted: List[Sequence] = []
        self.scheduled = set()


class Scheduler:
    def __init__(self, block_manager, max_num_seqs: int = 256, max_num_batched_tokens: int = 8192,
                 max_model_len: int = 8192, max_prefill_chunk: Optional[int] = None, policy: str = "prefill_first",
                 max_decode_stall: int = 4):
        self.bm = block_manager
        self.max_num_seqs = max_num_seqs
        self.max_num_batched_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.max_prefill_chunk = max_prefill_chunk or max_num_batched_tokens
        if policy not in ("prefill_first", "decode_first"):
            raise ValueError(f"unknown scheduling policy {policy!r}")
        self.policy = policy
        self.max_decode_stall = max_decode_stall
        self._decode_stall = 0
        self.waiting: Deque[Sequence] = collections.deque()
        self.running: List[Sequence] = []
        self.by_request: Dict[str, Sequence] = {}
        self.num_preemptions = 0
        self.prefix_caching = bool(getattr(block_manager, "prefix_caching", False))
        # seq_id -> (chained block hashes, prompt tokens) at admission
        self._hashes: Dict[int, Tuple[np.ndarray, np.ndarray]] = {}
        self.num_cached_tokens = 0  # prompt tokens served from the prefix cache

    # --------------------------------------------------------------- queue ops
    def add(self, seq: Sequence) -> None:
        if seq.num_tokens + seq.params.max_tokens > self.max_model_len + 1:
            # fail fast instead of overflowing the block table mid-generation
            room = self.max_model_len - seq.num_tokens
            if room < 1:
                raise ValueError(f"prompt of {seq.num_tokens} tokens exceeds max_model_len {self.max_model_len}")
            seq.params = dataclasses.replace(seq.params, max_tokens=room)
        if self.bm.blocks_for(seq.num_tokens + 1) > self.bm.num_blocks:
            raise ValueError("request can never fit in the KV cache")
        cap = self.bm.num_blocks * self.bm.block_size - seq.num_tokens
        if seq.params.max_tokens > cap:
            # a lone sequence must always be able to finish, or preemption would livelock
            seq.params = dataclasses.replace(seq.params, max_tokens=cap)
        self.waiting.append(seq)
        self.by_request[seq.request_id] = seq

    def abort(self, request_id: str) -> Optional[Sequence]:
        seq = self.by_request.pop(request_id, None)
        if seq is None:
            return None
        if seq in self.running:
            self.running.remove(seq)
        else:
            try:
                self.waiting.remove(seq)
            except ValueError:
                pass
        self.bm.free_seq(seq.seq_id)
        self._hashes.pop(seq.seq_id, None)
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = FinishReason.ABORT
        seq.finish_time = time.monotonic()
        return seq

    def finish(self, seq: Sequence, reason: FinishReason) -> None:
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        seq.finish_time = time.monotonic()
        self.bm.free_seq(seq.seq_id)
        self._hashes.pop(seq.seq_id, None)
        self.by_request.pop(seq.request_id, None)

    def remove_finished(self) -> None:
        self.running = [s for s in self.running if s.status != SeqStatus.FINISHED]

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def num_unfinished(self) -> int:
        return len(self.waiting) + len(self.running)

    # ------------------------------------------------------------ prefix cache
    def _match_prefix(self, seq: Sequence) -> None:
        """Admission of a sequence with nothing computed: reuse cached blocks of its prefix."""
        if not self.prefix_caching or seq.num_computed != 0 or self.bm.has(seq.seq_id):
            return
        bs = self.bm.block_size
        toks = np.asarray(seq.token_slice(0, seq.num_tokens), dtype=np.int32)
        h = self.bm.prefix_hashes(toks, salt=_salt(seq.cache_salt))
        self._hashes[seq.seq_id] = (h, toks)
        usable = max(0, (seq.num_tokens - 2) // bs)  # >= 2 tokens left: the step still samples
        got = self.bm.match_prefix(seq.seq_id, h, toks, min(usable, len(h)))
        seq.num_computed = got * bs

    def _unmatch(self, seq: Sequence) -> None:
        """Admission failed after a match: hand the blocks back (they stay cached)."""
        if self.prefix_caching and seq.num_computed and self.bm.has(seq.seq_id):
            self.bm.free_seq(seq.seq_id)
            seq.num_computed = 0

    def commit_prefix(self, seq: Sequence) -> None:
        """Register the sequence's full blocks whose KV is now in the cache."""
        ht = self._hashes.get(seq.seq_id)
        if ht is not None and not seq.is_finished():
            self.bm.commit_prefix(seq.seq_id, ht[0], ht[1], seq.num_computed // self.bm.block_size)

    # ------------------------------------------------------------------ policy
    def _preempt_youngest(self, protect: Sequence) -> Optional[Sequence]:
        """Free the youngest running sequence that is younger than ``protect``; None when
        ``protect`` is itself the youngest (it then yields instead: an older sequence is never
        evicted for a younger one, or two that do not fit together evict each other forever)."""
        if not self.running or self.running[-1] is protect:
            return None
        cand = self.running.pop()
        self.bm.free_seq(cand.seq_id)
        cand.num_computed = 0
        cand.status = SeqStatus.WAITING
        cand.num_preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(cand)
        return cand

    def schedule(self) -> ScheduledBatch:
        st = _Step(self.max_num_batched_tokens)
        # prefill-first: new prompts are admitted ahead of the running decodes (those run with
        # whatever budget is left), so a wave of prompts is prefilled in full budget-sized
        # steps with no decode rows mixed in -- GEMM shapes stay multiples of the budget and no
        # small tail chunk is left for an extra un-graphed step.  Decodes are skipped for at
        # most max_decode_stall consecutive steps, then a decode-first step runs.
        pf = (self.policy == "prefill_first" and bool(self.waiting) and bool(self.running)
              and self._decode_stall < self.max_decode_stall)
        if pf:
            self._admit(st)
        self._schedule_running(st)
        if not pf:
            self._admit(st)
        skipped = any(s.num_pending == 1 and s.seq_id not in st.scheduled for s in self.running)
        self._decode_stall = self._decode_stall + 1 if skipped else 0
        return ScheduledBatch(st.decodes, st.prefills, st.preempted)

    def _schedule_running(self, st: "_Step") -> None:
        i = 0
        while i < len(self.running) and st.budget > 0:
            seq = self.running[i]
            if seq.seq_id in st.scheduled:  # admitted earlier in this step (prefill-first)
                i += 1
                continue
            pending = seq.num_pending
            n = 1 if pending == 1 else min(pending, st.budget, self.max_prefill_chunk)
            while not self.bm.allocate(seq.seq_id, seq.num_computed + n):
                victim = self._preempt_youngest(protect=seq)
                if victim is None:
                    break
                st.preempted.append(victim)
            else:
                if pending == 1:
                    st.decodes.append(seq)
                else:
                    st.prefills.append((seq, n))
                st.scheduled.add(seq.seq_id)
                st.budget -= n
                i = self._index(seq) + 1  # preemption may have removed earlier entries
                continue
            # could not even fit this sequence alone: preempt it too
            i = self._index(seq)
            self.running.remove(seq)
            self.bm.free_seq(seq.seq_id)
            seq.num_computed = 0
            seq.status = SeqStatus.WAITING
            seq.num_preemptions += 1
            self.num_preemptions += 1
            self.waiting.appendleft(seq)
            st.preempted.append(seq)
        # preempted sequences that were already scheduled this step are dropped from it
        if st.preempted:
            gone = {s.seq_id for s in st.preempted}
            st.decodes = [s for s in st.decodes if s.seq_id not in gone]
            st.prefills = [(s, n) for s, n in st.prefills if s.seq_id not in gone]
            st.budget = self.max_num_batched_tokens - len(st.decodes) - sum(n for _, n in st.prefills)

    def _index(self, seq) -> int:
        """Position of ``seq`` in ``running`` (kept sorted by seq id): O(log n), not a scan."""
        return bisect.bisect_left(self.running, seq.seq_id, key=lambda s: s.seq_id)

    def _admit(self, st: "_Step") -> None:
        preempted = {s.seq_id for s in st.preempted}
        while self.waiting and st.budget > 0 and len(self.running) < self.max_num_seqs:
            seq = self.waiting[0]
            if seq.seq_id in preempted:
                break  # do not thrash: re-admit preempted sequences next step
            self._match_prefix(seq)
            n = min(seq.num_pending, st.budget, self.max_prefill_chunk)
            if not self.bm.can_allocate(seq.seq_id, seq.num_computed + n, True):
                self._unmatch(seq)
                break
            self.bm.allocate(seq.seq_id, seq.num_computed + n)
            self.waiting.popleft()
            seq.status = SeqStatus.RUNNING
            if seq.first_scheduled is None:
                # cache hits count once per request: a preempted sequence re-admitted later
                # re-matches its own committed blocks (prompt + output), which is no hit
                seq.first_scheduled = time.monotonic()
                seq.num_cached_tokens = min(seq.num_computed, len(seq.prompt_ids))
                self.num_cached_tokens += seq.num_cached_tokens
            # `running` stays in arrival order (seq ids are monotonic): a re-admitted preempted
            # sequence keeps its age, so "youngest" in _preempt_youngest is the latest arrival
            # (appending it made an old sequence the youngest and two sequences that do not fit
            # together could preempt each other forever under prefill_first)
            bisect.insort(self.running, seq, key=lambda s: s.seq_id)
            st.scheduled.add(seq.seq_id)
            if seq.num_pending == 1 and n == 1:
                st.decodes.append(seq)
            else:
                st.prefills.append((seq, n))
            st.budget -= n
