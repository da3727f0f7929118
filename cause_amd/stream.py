"""Streamed reweave of many batches of CausalLists from host memory (SURVEY
8(d) config 3: 10^6 documents processed in 10k-document batches).

The reference reweaves one collection at a time wherever a `weave-fn` runs
(list.cljc:26-28 via shared.cljc:259-266).  A host that holds far more
documents than one batch feeds the GPU here as a pipeline of `depth` slots:

    host fill (caller's producer, e.g. the generator, into pinned slot memory)
      -> H2D on the copy-in stream
      -> cw_weave_lists on the compute stream (the library's own kernels)
      -> D2H of weave_perm / visible bits / counts / max_ts / status on the
         copy-out stream
      -> the caller's consumer reads the pinned result of that slot

Batch i+1's H2D and batch i-1's D2H run under batch i's weave; the slot's
buffers are reused only after the events say the earlier batch is done with
them.  Every byte of node data is moved by DMA or touched by libcauseweave's
kernels; torch supplies device memory, pinned host memory, streams and events.
"""
from __future__ import annotations

import concurrent.futures as cf
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import abi


@dataclass
class BatchOut:
    """Pinned host view of one woven batch (valid inside the consumer call)."""
    index: int
    n_docs: int
    n_nodes: int
    weave_perm: np.ndarray      # u32[n_nodes] (u16 with perm16), doc-local input index
    visible_bits: np.ndarray    # u32[(n_nodes+31)//32]
    visible_count: np.ndarray   # u32[n_docs]
    max_ts: np.ndarray          # u64[n_docs]
    status: np.ndarray          # u32[n_docs]


@dataclass
class StreamStats:
    batches: int = 0
    nodes: int = 0
    wall_s: float = 0.0
    weave_ms: list = field(default_factory=list)    # per batch, compute-stream events
    h2d_ms: list = field(default_factory=list)
    d2h_ms: list = field(default_factory=list)
    fill_s: float = 0.0        # producer time (host fill), overlapped

    @property
    def device_nodes_per_s(self):
        t = sum(self.weave_ms) / 1e3
        return self.nodes / t if t else 0.0

    @property
    def end_to_end_nodes_per_s(self):
        return self.nodes / self.wall_s if self.wall_s else 0.0


class _Slot:
    def __init__(self, dev, max_nodes, max_docs, k32=False, perm16=False):
        pin = dict(pin_memory=True)
        kt = torch.int32 if k32 else torch.int64
        pt = torch.int16 if perm16 else torch.int32
        self.k32 = k32
        self.h_id = torch.empty(max_nodes, dtype=kt, **pin)
        self.h_ca = torch.empty(max_nodes, dtype=kt, **pin)
        self.h_kd = torch.empty(max_nodes, dtype=torch.uint8, **pin)
        nb = (max_nodes + 31) // 32
        self.h_perm = torch.empty(max_nodes, dtype=pt, **pin)
        self.h_bits = torch.empty(nb, dtype=torch.int32, **pin)
        self.h_vc = torch.empty(max_docs, dtype=torch.int32, **pin)
        self.h_mt = torch.empty(max_docs, dtype=torch.int64, **pin)
        self.h_st = torch.empty(max_docs, dtype=torch.int32, **pin)
        e = lambda n, t: torch.empty(n, dtype=t, device=dev)
        self.d_id, self.d_ca, self.d_kd = (e(max_nodes, kt), e(max_nodes, kt),
                                           e(max_nodes, torch.uint8))
        self.d_perm, self.d_bits = e(max_nodes, pt), e(nb, torch.int32)
        self.d_vc, self.d_mt, self.d_st = (e(max_docs, torch.int32), e(max_docs, torch.int64),
                                           e(max_docs, torch.int32))
        ev = lambda: torch.cuda.Event(enable_timing=True)
        self.ev_h2d0, self.ev_h2d, self.ev_w0, self.ev_w, self.ev_d2h0, self.ev_d2h = (
            ev(), ev(), ev(), ev(), ev(), ev())
        self.busy = None     # (batch index, n_docs, n_nodes) in flight
        self.offsets = None

    def host_inputs(self, n):
        """numpy views (id, cause: u64, or u32 for K32; kind u8) of the first n
        pinned input slots."""
        kt = np.uint32 if self.k32 else np.uint64
        return (self.h_id[:n].numpy().view(kt), self.h_ca[:n].numpy().view(kt),
                self.h_kd[:n].numpy())


class BatchStreamer:
    """Weave a sequence of host-resident batches through one GPU.

    fill(i, (id, cause, kind) pinned numpy views) -> offsets (u64[D+1]) fills
    batch i into the slot and returns its document offsets; it runs on a
    producer thread (`depth` - 1 batches ahead of the GPU).  consume(BatchOut)
    runs on the calling thread once the batch's results are in host memory.

    The streamer borrows the Weaver: while it is open the Weaver launches on
    the streamer's compute stream and returns right after enqueueing.  close()
    (or leaving a ``with`` block) gives the Weaver back on its own stream, in
    synchronous mode.

    k32: the slots hold 4-byte keys (cw_weave_lists_k32; fill writes u32 ids
    and causes, nil = abi.NIL32): 9 instead of 17 input bytes a node over PCIe.
    perm16 (with k32; documents < 65536 nodes): weave_perm comes back as u16."""

    def __init__(self, weaver: abi.Weaver, device, max_nodes, max_docs, layout, depth=2,
                 k32=False, perm16=False):
        if perm16 and not k32:
            raise ValueError("perm16 needs k32")
        if depth < 2:
            raise ValueError("depth >= 2")
        self.w = weaver
        self.dev = torch.device(device)
        self.layout = layout
        self.max_nodes, self.max_docs = int(max_nodes), int(max_docs)
        self.s_in = torch.cuda.Stream(self.dev)
        self.s_w = torch.cuda.Stream(self.dev)
        self.s_out = torch.cuda.Stream(self.dev)
        self.k32, self.perm16 = k32, perm16
        self.slots = [_Slot(self.dev, self.max_nodes, self.max_docs, k32, perm16)
                      for _ in range(depth)]
        weaver.set_stream(self.s_w.cuda_stream)
        weaver.set_async(True)
        self._open = True
        torch.cuda.synchronize(self.dev)

    def close(self):
        """Finish the streamer's work and hand the Weaver back (its own stream,
        synchronous calls)."""
        if getattr(self, "_open", False):
            torch.cuda.synchronize(self.dev)
            self.w.set_async(False)
            self.w.set_stream(None)
            self._open = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _fill(self, fill, i, slot):
        # the slot's pinned inputs are free once the previous H2D from them ran
        slot.ev_h2d.synchronize()
        t0 = time.perf_counter()
        n_cap = self.max_nodes
        off = np.ascontiguousarray(fill(i, slot.host_inputs(n_cap)), np.uint64)
        D, N = len(off) - 1, int(off[-1])
        if D < 1 or D > self.max_docs or N > n_cap or int(off[0]) != 0:
            raise ValueError(f"batch {i}: {D} documents / {N} nodes do not fit the slot "
                             f"({self.max_docs} / {n_cap})")
        return off, time.perf_counter() - t0

    def _launch(self, i, slot, off):
        D, N = len(off) - 1, int(off[-1])
        with torch.cuda.stream(self.s_in):
            self.s_in.wait_event(slot.ev_w)          # device inputs free (previous weave done)
            slot.ev_h2d0.record(self.s_in)
            slot.d_id[:N].copy_(slot.h_id[:N], non_blocking=True)
            slot.d_ca[:N].copy_(slot.h_ca[:N], non_blocking=True)
            slot.d_kd[:N].copy_(slot.h_kd[:N], non_blocking=True)
            slot.ev_h2d.record(self.s_in)
        self.s_w.wait_event(slot.ev_h2d)
        self.s_w.wait_event(slot.ev_d2h)             # device outputs free (previous D2H done)
        slot.ev_w0.record(self.s_w)
        outs = {"weave_perm": slot.d_perm.data_ptr(), "visible_bits": slot.d_bits.data_ptr(),
                "visible_count": slot.d_vc.data_ptr(), "max_ts": slot.d_mt.data_ptr(),
                "status": slot.d_st.data_ptr()}
        if self.k32:
            self.w.weave_lists_k32_device(off, slot.d_id.data_ptr(), slot.d_ca.data_ptr(),
                                          slot.d_kd.data_ptr(), self.layout, outs,
                                          perm16=self.perm16)
        else:
            self.w.weave_lists_device(off, slot.d_id.data_ptr(), slot.d_ca.data_ptr(),
                                      slot.d_kd.data_ptr(), self.layout, outs)
        slot.ev_w.record(self.s_w)
        nb = (N + 31) // 32
        with torch.cuda.stream(self.s_out):
            self.s_out.wait_event(slot.ev_w)
            slot.ev_d2h0.record(self.s_out)
            slot.h_perm[:N].copy_(slot.d_perm[:N], non_blocking=True)
            slot.h_bits[:nb].copy_(slot.d_bits[:nb], non_blocking=True)
            slot.h_vc[:D].copy_(slot.d_vc[:D], non_blocking=True)
            slot.h_mt[:D].copy_(slot.d_mt[:D], non_blocking=True)
            slot.h_st[:D].copy_(slot.d_st[:D], non_blocking=True)
            slot.ev_d2h.record(self.s_out)
        slot.busy = (i, D, N)
        slot.offsets = off

    def _retire(self, slot, consume, stats):
        i, D, N = slot.busy
        slot.ev_d2h.synchronize()
        stats.h2d_ms.append(slot.ev_h2d0.elapsed_time(slot.ev_h2d))
        stats.weave_ms.append(slot.ev_w0.elapsed_time(slot.ev_w))
        stats.d2h_ms.append(slot.ev_d2h0.elapsed_time(slot.ev_d2h))
        stats.batches += 1
        stats.nodes += N
        if consume is not None:
            consume(BatchOut(i, D, N, slot.h_perm[:N].numpy().view(
                             np.uint16 if self.perm16 else np.uint32),
                             slot.h_bits[:(N + 31) // 32].numpy().view(np.uint32),
                             slot.h_vc[:D].numpy().view(np.uint32),
                             slot.h_mt[:D].numpy().view(np.uint64),
                             slot.h_st[:D].numpy().view(np.uint32)))
        slot.busy = None

    def run(self, n_batches, fill, consume=None) -> StreamStats:
        stats = StreamStats()
        S = len(self.slots)
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(1) as ex:
            futs = {}
            for j in range(min(S - 1, n_batches)):
                futs[j] = ex.submit(self._fill, fill, j, self.slots[j % S])
            for i in range(n_batches):
                slot = self.slots[i % S]
                if slot.busy is not None:       # batch i-S: results to the consumer
                    self._retire(slot, consume, stats)
                off, t_fill = futs.pop(i).result()
                stats.fill_s += t_fill
                # the producer starts on batch i+S-1 before batch i is launched
                # (a launch may block the host: profiling syncs every weave); its
                # slot's inputs are rewritten once that slot's H2D has run
                nxt = i + S - 1
                if nxt < n_batches:
                    futs[nxt] = ex.submit(self._fill, fill, nxt, self.slots[nxt % S])
                self._launch(i, slot, off)
            for k in range(max(0, n_batches - S), n_batches):   # drain in batch order
                s = self.slots[k % S]
                if s.busy is not None and s.busy[0] == k:
                    self._retire(s, consume, stats)
        torch.cuda.synchronize(self.dev)
        stats.wall_s = time.perf_counter() - t0
        return stats
