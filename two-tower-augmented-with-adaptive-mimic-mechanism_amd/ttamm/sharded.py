"""Row-sharded multi-GPU training step (one process per GPU, RCCL over xGMI).

The reference trains on one device (training.py:1243-1244); a W-rank step here is defined as
the reference's step over the GLOBAL batch formed by concatenating the ranks' batches
(rank-major).  Each rank owns

  * users u with u % W == rank (local row u // W): ID + mimic rows, feature rows, positives;
    a rank's batch holds only its own users, so the user side needs no exchange;
  * items i with i % W == rank (local row i // W): ID + mimic rows and feature rows; the item
    tower of an item runs on its owner for whoever requested it;
  * a replica of the feature-encoder / gate weights (all-reduced gradients).

Per step (ttamm.h TTAMM_PHASE_*):

  SAMPLE    negatives for the rank's users, from the global item range
  a2a       requested item ids + their global request positions -> owners
  ITEM_FWD  owner: item tower over the requested rows            -> (t | a) rows
  a2a       (t | a) rows -> requesters               (overlaps USER_FWD on the GPU)
  USER_FWD  user tower
  (in-batch negatives only: INBATCH_SRC -> all-gather of the ranks' augmented positives
   [B, D] -> [W B, D] -> INBATCH: S = U P^T over the global batch -> reduce-scatter of dP)
  USER      scores, losses, user backward + user-table updates   -> (dT | dA) rows
  a2a       (dT | dA) rows -> owners
  ITEM_BWD  owner: item backward + item-table updates
  allreduce replicated-weight gradients (+ this rank's loss share, same buffer)
  DENSE     AdamW on the replicated weights

Negative sampling and dropout draw from Philox streams keyed by global positions, so the W
ranks draw exactly what one process would for the global batch; losses are normalised by the
global batch.  Every rank sweeps AdamW(g=0) over its own table shards only.

The step is written as an SPMD program that yields a request at each collective.
``TorchComm`` serves the requests with torch.distributed (RCCL on ROCm, gloo on CPU);
``run_loopback`` runs W programs in one process in lock step (the single-GPU parity test).
"""

from __future__ import annotations

import ctypes
import functools
import os
from dataclasses import dataclass, field
from typing import Any, Callable, Generator, Mapping, Sequence

import torch

from . import _lib
from .training import FusedTrainStep


# ---------------------------------------------------------------------------------------
# ownership
# ---------------------------------------------------------------------------------------
@dataclass(frozen=True)
class RowOwnership:
    """Row i of a table lives on rank i % world_size at local row i // world_size."""

    world_size: int
    rank: int

    def __post_init__(self) -> None:
        if self.world_size < 1 or not 0 <= self.rank < self.world_size:
            raise ValueError("ttamm: bad (world_size, rank)")

    def local_count(self, rows: int) -> int:
        return max(0, (rows - self.rank + self.world_size - 1) // self.world_size)

    def owner(self, ids: torch.Tensor) -> torch.Tensor:
        return torch.remainder(ids, self.world_size)

    def local(self, ids: torch.Tensor) -> torch.Tensor:
        return torch.div(ids, self.world_size, rounding_mode="floor")

    def global_ids(self, local_rows: torch.Tensor) -> torch.Tensor:
        return local_rows * self.world_size + self.rank

    def shard(self, full: torch.Tensor) -> torch.Tensor:
        """This rank's rows of a global table (a copy, contiguous)."""
        return full[self.rank :: self.world_size].contiguous()

    def local_padding_idx(self, padding_idx: int | None) -> int | None:
        """The shard's nn.Embedding padding_idx for a table whose global padding row is
        ``padding_idx`` (encoders.py:47): its local row on the owner, None on every other rank."""
        if padding_idx is None or int(padding_idx) % self.world_size != self.rank:
            return None
        return int(padding_idx) // self.world_size


# ---------------------------------------------------------------------------------------
# collectives as requests
# ---------------------------------------------------------------------------------------
@dataclass
class AllToAll:
    """Rows of ``send`` grouped by destination (``send_splits`` rows each) -> rows grouped by
    source (``recv_splits`` rows each)."""

    send: torch.Tensor
    send_splits: list[int]
    recv_splits: list[int]
    async_op: bool = False
    out: torch.Tensor | None = None  # receive buffer (sum(recv_splits) rows); None = a new tensor


@dataclass
class Wait:
    handle: Any


@dataclass
class AllReduce:
    """In-place sum over ranks."""

    tensor: torch.Tensor


@dataclass
class AllGather:
    """Every rank's ``send`` (same shape on all ranks), concatenated rank-major."""

    send: torch.Tensor


@dataclass
class ReduceScatter:
    """``send`` holds W equal chunks along dim 0; rank r gets the sum over ranks of chunk r."""

    send: torch.Tensor


Program = Generator[Any, Any, Any]


class TorchComm:
    """Serves a program's requests with torch.distributed (backend "nccl" is RCCL on ROCm).
    With a gloo group, device tensors are staged through host memory (gloo moves CPU tensors
    only) — for tests that put several ranks on one GPU, which RCCL does not allow."""

    def __init__(self, group: Any = None) -> None:
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.staged = dist.get_backend(group) == "gloo"

    def __call__(self, req: Any) -> Any:
        dist = self.dist
        if isinstance(req, AllToAll):
            send = req.send.contiguous()
            dev = send.device
            if self.staged:
                send = send.cpu()
            out = send.new_empty((sum(req.recv_splits),) + tuple(send.shape[1:]))
            if self.staged:
                dist.all_to_all_single(out, send, req.recv_splits, req.send_splits, group=self.group)
                out = out.to(dev) if req.out is None else req.out.copy_(out)
                return (None, out) if req.async_op else out
            if req.out is not None:
                out = req.out
            work = dist.all_to_all_single(out, send, req.recv_splits, req.send_splits,
                                          group=self.group, async_op=req.async_op)
            return (work, out) if req.async_op else out
        if isinstance(req, Wait):
            work, out = req.handle
            if work is not None:
                work.wait()
            return out
        if isinstance(req, AllGather):
            send = req.send.contiguous()
            W = dist.get_world_size(self.group)
            if self.staged:
                host = send.cpu()
                out = host.new_empty((W * host.shape[0],) + tuple(host.shape[1:]))
                dist.all_gather(list(out.chunk(W)), host, group=self.group)
                return out.to(send.device)
            out = send.new_empty((W * send.shape[0],) + tuple(send.shape[1:]))
            dist.all_gather_into_tensor(out, send, group=self.group)
            return out
        if isinstance(req, ReduceScatter):
            send = req.send.contiguous()
            W = dist.get_world_size(self.group)
            if self.staged:  # gloo has no reduce-scatter: all-reduce the host copy, keep this rank's chunk
                host = send.cpu()
                dist.all_reduce(host, group=self.group)
                return host.chunk(W)[dist.get_rank(self.group)].contiguous().to(send.device)
            out = send.new_empty((send.shape[0] // W,) + tuple(send.shape[1:]))
            dist.reduce_scatter_tensor(out, send, group=self.group)
            return out
        if isinstance(req, AllReduce):
            if self.staged and req.tensor.device.type != "cpu":
                host = req.tensor.cpu()
                dist.all_reduce(host, group=self.group)
                req.tensor.copy_(host)
            else:
                dist.all_reduce(req.tensor, group=self.group)
            return req.tensor
        raise TypeError(f"unknown collective request {req!r}")

    def run(self, program: Program) -> Any:
        res = None
        try:
            while True:
                res = self(program.send(res))
        except StopIteration as stop:
            return stop.value


class MirrorComm:
    """Serves ONE rank's collectives as if the other W - 1 ranks ran the same program on the same
    data relabelled (rank s's traffic to rank d is this rank's traffic to rank d - s + rank):
    an all-to-all returns this rank's own send chunks (the chunk "from" rank s is the one this
    rank sends to rank 2 rank - s, so every split agrees with the count exchange), an
    all-gather W copies of ``send``, a reduce-scatter this rank's chunk, an all-reduce the tensor
    unchanged.  The rank then does exactly the per-rank work of a W-rank step — W x its own
    item requests as owner, the W B-row all-gathered in-batch positives — with no interconnect
    traffic.  A measurement device (``bench.py --emulate-world``), not a numerically meaningful
    run: the values are not those of any W-rank job."""

    def __init__(self, world_size: int, rank: int = 0) -> None:
        if world_size < 1 or not 0 <= rank < world_size:
            raise ValueError("ttamm: bad (world_size, rank)")
        self.world, self.rank = int(world_size), int(rank)

    def __call__(self, req: Any) -> Any:
        W, me = self.world, self.rank
        if isinstance(req, AllToAll):
            chunks = list(torch.split(req.send, req.send_splits))
            parts = [chunks[(2 * me - s) % W] for s in range(W)]
            if sum(p.shape[0] for p in parts) != sum(req.recv_splits):
                raise RuntimeError("mirror: recv splits do not match the mirrored sends")
            # one pass into the receive buffer, as an all-to-all writes it
            got = torch.cat(parts, out=req.out) if req.out is not None else torch.cat(parts)
            return (None, got) if req.async_op else got
        if isinstance(req, Wait):
            return req.handle[1]
        if isinstance(req, AllGather):
            return torch.cat([req.send] * W)
        if isinstance(req, ReduceScatter):
            return req.send.chunk(W)[me].contiguous()
        if isinstance(req, AllReduce):
            return req.tensor
        raise TypeError(f"unknown collective request {req!r}")

    def run(self, program: Program) -> Any:
        res = None
        try:
            while True:
                res = self(program.send(res))
        except StopIteration as stop:
            return stop.value


def run_loopback(programs: Sequence[Program]) -> list[Any]:
    """Run W SPMD programs in one process, serving their collectives jointly.  Rank order is
    the reduction order of AllReduce (fixed, deterministic)."""
    W = len(programs)
    results: list[Any] = [None] * W
    done: list[bool] = [False] * W
    values: list[Any] = [None] * W
    while not all(done):
        reqs: list[Any] = [None] * W
        for r, prog in enumerate(programs):
            if done[r]:
                continue
            try:
                reqs[r] = prog.send(results[r])
            except StopIteration as stop:
                done[r] = True
                values[r] = stop.value
        if all(done):
            break
        if any(done):
            raise RuntimeError("loopback: ranks issued different collective sequences")
        kind = type(reqs[0])
        if any(type(q) is not kind for q in reqs):
            raise RuntimeError("loopback: ranks issued different collectives")
        if kind is AllToAll:
            chunks = [list(torch.split(q.send, q.send_splits)) for q in reqs]
            for d in range(W):
                got = torch.cat([chunks[s][d] for s in range(W)])
                if got.shape[0] != sum(reqs[d].recv_splits):
                    raise RuntimeError("loopback: recv splits do not match the senders")
                if reqs[d].out is not None:
                    got = reqs[d].out.copy_(got)
                results[d] = ("done", got) if reqs[d].async_op else got
        elif kind is Wait:
            for r in range(W):
                results[r] = reqs[r].handle[1]
        elif kind is AllReduce:
            total = reqs[0].tensor.clone()
            for r in range(1, W):
                total += reqs[r].tensor
            for r in range(W):
                reqs[r].tensor.copy_(total)
                results[r] = reqs[r].tensor
        elif kind is AllGather:
            got = torch.cat([q.send for q in reqs])
            for r in range(W):
                results[r] = got.clone()
        elif kind is ReduceScatter:
            total = reqs[0].send.clone()
            for r in range(1, W):
                total += reqs[r].send
            for r, chunk in enumerate(total.chunk(W)):
                results[r] = chunk.contiguous()
        else:
            raise TypeError(f"unknown collective request {reqs[0]!r}")
    return values


# ---------------------------------------------------------------------------------------
# request routing
# ---------------------------------------------------------------------------------------
@dataclass
class Route:
    slot: torch.Tensor  # request position -> its row in the owner-grouped exchange buffers
    send_counts: list[int]  # requests to each owner
    recv_counts: list[int]  # requests from each requester
    rows: torch.Tensor  # owner side: local rows requested [n_recv]
    keys: torch.Tensor  # owner side: global request positions [n_recv]
    own_status: int = 0  # this rank's status word after SAMPLE (when piggybacked)
    peer_status: int = 0  # OR of the other ranks' status words
    # compact exchange rows (count rows with a positives column): of send_counts / recv_counts,
    # the leading positives; sr = the device count rows [2W, ld] (ttamm_step_args.exchange_counts)
    send_pos: list[int] = field(default_factory=list)
    recv_pos: list[int] = field(default_factory=list)
    sr: torch.Tensor | None = None


def device_route(lib: Any, world: int, id0: torch.Tensor, id1: torch.Tensor | None = None,
                 payload: torch.Tensor | None = None, key0: int = 0, key1: int = 0,
                 counts_out: torch.Tensor | None = None,
                 status: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """ttamm_route_rows: ids [id0; id1] grouped by owner (id % world), stably.  Returns (packed
    [n, 2] = (id // world, payload or key) in the grouped order, slot [n], counts [world]).
    ``counts_out`` may be a [world, 2] int64 buffer: column 0 gets the counts and, with ``status``
    (the int32 status word), column 1 the status — the count all-to-all's send rows, one launch."""
    dev = id0.device
    n0 = id0.numel()
    n1 = id1.numel() if id1 is not None else 0
    n = n0 + n1
    packed = torch.empty((n, 2), dtype=torch.long, device=dev)
    slot = torch.empty(n, dtype=torch.long, device=dev)
    counts = counts_out if counts_out is not None else torch.empty(world, dtype=torch.long, device=dev)
    ld = counts.stride(0) if counts.dim() == 2 else 1
    scratch = torch.empty(max(1, int(lib.ttamm_route_scratch_bytes(n, world))), dtype=torch.uint8, device=dev)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else None  # noqa: E731
    _lib.check(lib.ttamm_route_rows(ptr(id0), n0, ptr(id1), n1, ptr(payload), key0, key1, world, ptr(packed),
                                    ptr(slot), ctypes.c_void_p(counts.data_ptr()), ld, ptr(status),
                                    ctypes.c_void_p(scratch.data_ptr()), scratch.numel(), _lib.stream_handle(dev)))
    return packed, slot, counts


Router = Callable[..., "tuple[torch.Tensor, torch.Tensor, torch.Tensor]"]  # device_route minus lib


@dataclass
class PendingRoute:
    """route_start's result: the requests grouped by owner, the count rows exchanged, their copy
    to the host in flight (``event`` marks it)."""

    packed: torch.Tensor
    slot: torch.Tensor
    n: int
    sr: torch.Tensor  # [2W, ld] (count, status[, positives]) rows sent, then received
    host: torch.Tensor | None  # pinned copy of sr (None: read sr itself)
    event: Any  # torch.cuda.Event after the copy, or None


def route_start(own: RowOwnership, router: Router, pos: torch.Tensor, negs: torch.Tensor, key0: int, key1: int,
                status: torch.Tensor | None = None, host: torch.Tensor | None = None, ld: int = 2) -> Program:
    """Program: group the requests [pos; negs] by owner (keys key0 + j for positives, key1 + j for
    negatives) and exchange the per-owner counts with the rank's status word (``ld`` = 3: and how
    many of them are positives, for the compact exchange rows).  With a pinned ``host`` buffer the
    counts are copied to it asynchronously (no host synchronisation here: route_finish waits, so a
    look-ahead can start the copy a step early)."""
    W = own.world_size
    n = pos.numel() + negs.numel()
    # rows 0..W-1: what this rank sends (count to owner d, its status word[, positives]); rows
    # W..2W-1: received
    sr = torch.empty((2 * W, ld), dtype=torch.long, device=pos.device)
    if status is None:
        sr[:W, 1] = 0
    packed, slot, _ = router(W, pos, negs, None, key0, key1, counts_out=sr[:W], status=status)
    event = None
    if W == 1 and ld >= 3:  # the owner's rows are this rank's own requests
        sr[1:].copy_(sr[:1])
    if W > 1:
        yield AllToAll(sr[:W], [1] * W, [1] * W, out=sr[W:])
        if host is not None and sr.device.type == "cuda":
            host.copy_(sr, non_blocking=True)
            event = torch.cuda.Event()
            event.record()
        else:
            host = None
    return PendingRoute(packed, slot, n, sr, host, event)


def route_finish(own: RowOwnership, pend: PendingRoute) -> Program:
    """Program: read the exchanged counts (the step's one host synchronisation, already done when
    a look-ahead started it a step earlier) and send (local row, key) of every request to its owner.
    Returns a Route.  The status words that rode with the counts tell every rank whether any rank's
    step is poisoned (Route.peer_status) before any of them writes state."""
    W = own.world_size
    ld = pend.sr.shape[1]
    if W == 1:  # (local row, key) columns read in place by the step (ttamm_step_args.item_rows_ld)
        # (no exchange: the positives' count stays on the device, in sr, for the step's unit maps)
        return Route(pend.slot, [pend.n], [pend.n], pend.packed[:, 0], pend.packed[:, 1], sr=pend.sr)
    if pend.host is not None:
        pend.event.synchronize()
        c = pend.host.reshape(-1).tolist()
    else:
        c = pend.sr.reshape(-1).tolist()
    sent, got_c = c[0:ld * W:ld], c[ld * W::ld]
    peers = 0
    for r, st in enumerate(c[ld * W + 1::ld]):
        if r != own.rank:
            peers |= int(st)
    got = yield AllToAll(pend.packed, sent, got_c)
    route = Route(pend.slot, sent, got_c, got[:, 0], got[:, 1], int(c[1]), peers, sr=pend.sr)
    if ld >= 3:
        route.send_pos, route.recv_pos = c[2:ld * W:ld], c[ld * W + 2::ld]
    return route


def route_requests(own: RowOwnership, router: Router, pos: torch.Tensor, negs: torch.Tensor, key0: int,
                   key1: int, status: torch.Tensor | None = None) -> Program:
    """Program: send (local row, key) of every requested item ([pos; negs], keys key0 + j for
    positives, key1 + j for negatives) to its owner.  Returns a Route.  One host sync (the
    counts, which size the variable all-to-all); none at world size 1.  ``status`` (the rank's
    device status word): rides along with the counts, so every rank learns whether any rank's
    step is poisoned (Route.peer_status) before any of them writes state."""
    pend = yield from route_start(own, router, pos, negs, key0, key1, status=status)
    return (yield from route_finish(own, pend))


# ---------------------------------------------------------------------------------------
# the sharded step
# ---------------------------------------------------------------------------------------
@dataclass
class _Ahead:
    """The next step as a look-ahead prepared it: its batch (matched by identity), negatives,
    status word and the request routing up to the exchanged counts."""

    users: torch.Tensor
    pos: torch.Tensor
    negs: torch.Tensor
    status: torch.Tensor
    pending: PendingRoute


class ShardedTrainStep(FusedTrainStep):
    """FusedTrainStep over a rank's shard.  ``model`` holds this rank's rows of the user / item
    ID and mimic tables (``RowOwnership.shard``) and a replica of the feature-encoder and gate
    weights; ``user_features`` / ``item_features`` are this rank's rows; ``positives`` is
    keyed by LOCAL user row and holds GLOBAL item ids; ``num_items`` is the global item count.

    Every rank must call ``step`` with the same batch size (the global batch is W x B, rank r's
    interactions are global positions [r B, (r+1) B)); ``step`` and ``finish`` are collective.

    Reference options (encoders.py:47-58, training.py:824-825):
      * padding_idx: the shard's ID table carries the padding row as a LOCAL row on its owner
        only (``RowOwnership.local_padding_idx``); it gets no gradient there, as in one process;
      * max_norm (dense ID tables): the owner renorms the rows looked up for every requester's
        positives, then for their negatives — the reference's two item lookups (training.py:750,
        :776) — and each rank its own users;
      * gradient_clip_norm (dense ID tables, grouped schedule): the table updates wait for the
        global norm — each rank's share over the table rows it owns rides in the gradient
        all-reduce (TTAMM_PHASE_TABLES), so every rank applies clip_grad_norm_'s one coefficient.
    """

    def __init__(self, model, optimizers, *, world_size: int, rank: int, num_items: int,
                 comm: Callable[[Program], Any] | None = None, group_towers: bool = True, **kw: Any) -> None:
        clip = kw.get("gradient_clip_norm")
        if clip is not None and clip > 0 and not group_towers:
            raise NotImplementedError("ttamm: gradient clipping in the row-sharded step needs group_towers=True")
        self.own = RowOwnership(world_size, rank)
        self.comm = comm
        # True: both towers' forward in one set of grouped launches, then the (t | a) exchange;
        # False: the item forward, the exchange overlapping the user forward, then the rest
        # (backward: score, exchange, then both towers' backward grouped / the user backward
        # first).  The grouped schedule launches each tower-wide kernel once per step.
        self.group_towers = bool(group_towers)
        self.item_rows_seen = 0  # item-tower rows this owner ran (bench roofline)
        # look-ahead routing (program(next_batch=...)): the prepared next step, its buffers
        self._ahead: _Ahead | None = None
        self._ahead_bufs: list[torch.Tensor] | None = None
        self._ahead_status: list[torch.Tensor] = []
        self._ahead_host: torch.Tensor | None = None
        self._ahead_flip = 0
        super().__init__(model, optimizers, num_items=num_items, **kw)
        self.router: Router = functools.partial(device_route, self.lib)

    def _configure(self, args: _lib.StepArgs) -> None:
        W = self.own.world_size
        R = self.max_batch * (1 + self.num_neg)
        # worst case: every requester sends all its rows to this owner
        self.capacity = W * R
        args.phase = _lib.PHASE_SAMPLE  # any non-zero phase: size the sharded workspace
        args.item_rows_capacity = self.capacity
        args.num_items_global = self.num_items
        n_grad = int(self.lib.ttamm_dense_grad_floats(ctypes.byref(args)))
        # gradient arena + this rank's loss share (+ its table-row squared gradient norm when
        # clipping): one all-reduce carries them all
        self.arena = torch.zeros(n_grad + 6, dtype=torch.float32, device=self.device)  # + loss_out[5] + sumsq
        self.n_grad = n_grad
        self.loss_out = self.arena[n_grad:n_grad + 5]
        self.clip = args.hp.grad_clip_norm > 0
        args.loss_out = self.loss_out.data_ptr()
        args.table_sumsq = self.arena[n_grad + 5:].data_ptr()
        args.dense_grads = self.arena.data_ptr()
        D = self.model.user_encoder.output_dim  # the tower output (= embedding dim unless concat sets another)
        self.D = D
        self.fwd_out = torch.empty((self.capacity, 2 * D), dtype=torch.float32, device=self.device)
        if self.in_batch:  # all-gathered positives: the workspace is sized for the global batch
            args.global_batch = W * self.max_batch
            self.ib_local = torch.empty((self.max_batch, D), dtype=torch.float32, device=self.device)
            self.ib_dp_all = torch.empty((W * self.max_batch, D), dtype=torch.float32, device=self.device)
        self.cal = self.item_categories is not None
        if self.cal:  # the global per-category sums / scatters (TTAMM_PHASE_CAL_*), all-reduced
            ncat = int(args.num_categories)
            self.cal_stats = torch.zeros(ncat * (D + 1), dtype=torch.float32, device=self.device)
            self.cal_scatter = torch.zeros(ncat * D * D, dtype=torch.float32, device=self.device)
            args.cal_stats = self.cal_stats.data_ptr()
            args.cal_scatter = self.cal_scatter.data_ptr()
        self.fwd_in = torch.empty((R, 2 * D), dtype=torch.float32, device=self.device)
        self.bwd_out = torch.empty((R, 2 * D), dtype=torch.float32, device=self.device)
        # compact exchange rows (ttamm.h ttamm_step_args.exchange_counts): a negative request moves D
        # floats each way instead of 2 D (t + a forward, dT backward); TTAMM_WIDE_EXCHANGE=1 keeps the
        # 2 D-wide rows.  The buffers above stay sized for the wide rows (the compact ones fit).  Without
        # sampled negatives (in-batch only, num_neg = 0) every request is a positive and the layouts
        # move the same bytes: the wide one is kept (no unit maps).
        self.compact = (self.num_neg > 0 and bool(self.lib.ttamm_exchange_compact_supported(ctypes.byref(args)))
                        and os.environ.get("TTAMM_WIDE_EXCHANGE") != "1")
        self.count_ld = 3 if self.compact else 2
        self.exchange_floats = [0, 0]  # this rank's last (t | a) send, (dT | dA) send, in floats

    def _phase(self, bits: int) -> None:
        self.args.phase = bits
        _lib.check(self.lib.ttamm_train_step(ctypes.byref(self.args), _lib.stream_handle(self.device)))

    def program(self, users: torch.Tensor, pos_items: torch.Tensor, neg_items: torch.Tensor | None = None, *,
                keep_masks: Mapping[str, Sequence[torch.Tensor]] | None = None,
                timing_events: Sequence[Any] | None = None, row_base: int | None = None,
                global_batch: int | None = None,
                next_batch: tuple[torch.Tensor, torch.Tensor] | None = None) -> Program:
        """One step as an SPMD program (yields collective requests).  ``timing_events``
        (hipEvent_t handles, pairs as in ttamm.h) bracket the owner's item-table maintenance
        and its item-tower first-layer GEMM.  By default every rank holds B interactions and
        rank r's are global positions [r B, (r + 1) B); ranks with different batch sizes pass
        ``row_base`` (the sizes of the ranks before this one) and ``global_batch`` (the sum).

        ``next_batch`` = (users, positives) of the following step (default positions, sampled
        negatives): its negatives are drawn, its requests grouped and its request counts
        exchanged during this step, after the forward exchange, and their copy to the host runs
        behind this step's backward — so the next step reads them without waiting (look-ahead
        routing; the draws and ids are the ones that step would make itself)."""
        ahead = self._ahead
        self._ahead = None
        mismatch = False
        if ahead is not None:
            # A prepared look-ahead already exchanged this step's request counts on EVERY rank, so
            # every rank consumes it (the same collective sequence everywhere, whatever this call
            # passes).  A call with another batch is a caller error: this rank's step is then
            # skipped (status bit, no state written) and finish() raises on every rank.
            same = (ahead.users is users and ahead.pos is pos_items) or (
                users.shape == ahead.users.shape and pos_items.shape == ahead.pos.shape
                and torch.equal(users, ahead.users) and torch.equal(pos_items, ahead.pos))
            mismatch = not same or neg_items is not None or row_base is not None or global_batch is not None
            users, pos_items, neg_items, row_base, global_batch = ahead.users, ahead.pos, None, None, None
        use_ahead = ahead is not None
        # the look-ahead runs at default positions only, decided on the EFFECTIVE row_base /
        # global_batch (after a prepared look-ahead replaced the caller's); its batch is validated
        # here, before this step's first collective, so a bad next_batch raises on this rank before
        # any other rank can wait on it
        look_ahead = next_batch is not None and row_base is None and global_batch is None
        if look_ahead:
            self._check_next_batch(*next_batch)
        if self.compact and not self.lib.ttamm_exchange_compact_supported(ctypes.byref(self.args)):
            # the compact layout was chosen at construction for the fused gate kernels; the gate
            # path is read from TTAMM_GENERIC_GATE on every step: say so up front,
            # before this step's first collective, instead of failing inside the step
            raise ValueError("ttamm: the gate path changed (TTAMM_GENERIC_GATE) after this sharded step was built "
                             "with compact exchange rows; build a new ShardedTrainStep")
        if not self._bind_batch(users, pos_items, ahead.negs if use_ahead else neg_items, keep_masks):
            raise ValueError("ttamm: empty batch in a sharded step (every rank must step)")
        a = self.args
        W, rank = self.own.world_size, self.own.rank
        B, N, D = users.numel(), self.num_neg, self.D
        Bg = W * B if global_batch is None else int(global_batch)
        base = rank * B if row_base is None else int(row_base)
        if self.in_batch and Bg != W * B:
            raise ValueError("ttamm: in-batch negatives need the same batch size on every rank")
        a.row_base = base
        a.global_batch = Bg
        nev = len(a.timing_events)
        ev = list(timing_events or []) + [None] * nev
        for i in range(nev):
            a.timing_events[i] = None
        self._hparams()
        if use_ahead:
            negs = ahead.negs
            self.status.bitwise_or_(ahead.status)  # what the look-ahead's checks and draws found
            if mismatch:
                self.status.bitwise_or_(_lib.STATUS_LOOKAHEAD_MISMATCH)
        else:
            negs = neg_items.reshape(-1) if neg_items is not None else self.neg_buffer[: B * N]
        self._phase(_lib.PHASE_SAMPLE)
        # ---- route the item requests [positives; negatives] to their owners -----------------
        if use_ahead:
            pend = ahead.pending
        else:
            pend = yield from route_start(self.own, self.router, pos_items.reshape(-1), negs, base, Bg + base * N,
                                          status=self.status, ld=self.count_ld)
        route = yield from route_finish(self.own, pend)
        if route.peer_status and not route.own_status:
            # another rank's step is poisoned (an id outside its table, sampler exhaustion):
            # poison this rank's step too, before it writes any state, so every rank keeps the
            # state after the same last good step; SAMPLE already counted the step here
            self.status.bitwise_or_(route.peer_status & _lib.STATUS_POISON)
            self.steps_applied.sub_(1)
        n = route.rows.numel()
        self.item_rows_seen += n
        if n > self.capacity:
            raise RuntimeError("ttamm: item requests exceed the sharded step's capacity")
        if route.rows.stride(0) != route.keys.stride(0):
            raise RuntimeError("ttamm: request rows and keys must share one stride")
        a.item_rows = route.rows.data_ptr()
        a.item_row_keys = route.keys.data_ptr()
        a.item_rows_ld = route.rows.stride(0) if n > 0 else 1
        a.n_item_rows = n
        a.item_slot = route.slot.data_ptr()  # exchange buffers stay in owner-grouped order
        a.item_fwd_out = self.fwd_out.data_ptr()
        R = B * (1 + N)
        if self.compact:
            # D-float units, a positive taking two: per peer D (requests + positives) floats each way
            a.exchange_counts = route.sr.data_ptr()
            a.exchange_counts_ld = route.sr.stride(0)
            a.exchange_world = W
            if W > 1:
                to_req = [D * (c + p) for c, p in zip(route.recv_counts, route.recv_pos)]
                to_own = [D * (c + p) for c, p in zip(route.send_counts, route.send_pos)]
                fwd_src = self.fwd_out.view(-1)[:sum(to_req)]
                fwd_dst = self.fwd_in.view(-1)[:sum(to_own)]
                bwd_src = self.bwd_out.view(-1)[:sum(to_own)]
        else:
            a.exchange_counts = None
            a.exchange_counts_ld = 0
            a.exchange_world = 0
            to_req, to_own = route.recv_counts, route.send_counts
            fwd_src, fwd_dst, bwd_src = self.fwd_out[:n], self.fwd_in[:R], self.bwd_out[:R]
        for i in (2, 3, 8, 9, 10, 11):  # first-layer GEMM, catch-up replays
            a.timing_events[i] = ev[i]
        if W == 1:  # no exchange: the requester's buffers are the owner's
            self._phase(_lib.PHASE_ITEM_FWD | _lib.PHASE_USER_FWD if self.group_towers else _lib.PHASE_ITEM_FWD)
            if not self.group_towers:
                self._phase(_lib.PHASE_USER_FWD)
            back = self.fwd_out[:n]
        elif self.group_towers:
            self._phase(_lib.PHASE_ITEM_FWD | _lib.PHASE_USER_FWD)
            self.exchange_floats[0] = fwd_src.numel()
            back = yield AllToAll(fwd_src, to_req, to_own, out=fwd_dst)
        else:  # (t | a) back to the requesters, the user tower meanwhile
            self._phase(_lib.PHASE_ITEM_FWD)
            self.exchange_floats[0] = fwd_src.numel()
            h = yield AllToAll(fwd_src, to_req, to_own, async_op=True, out=fwd_dst)
            self._phase(_lib.PHASE_USER_FWD)
            back = yield Wait(h)
        for i in (2, 3, 8, 9, 10, 11):
            a.timing_events[i] = None
        a.item_fwd_in = back.data_ptr()
        a.item_bwd_out = self.bwd_out.data_ptr()
        if look_ahead:
            self._ahead = yield from self._look_ahead(*next_batch)
        ib = ()
        if self.in_batch:
            # ---- in-batch: every rank's augmented positives, then dP summed back to its rank ------
            a.inbatch_local = self.ib_local.data_ptr()
            self._phase(_lib.PHASE_INBATCH_SRC)
            gathered = yield AllGather(self.ib_local[:B])
            a.inbatch_items = gathered.data_ptr()
            a.inbatch_dp_all = self.ib_dp_all.data_ptr()
            a.timing_events[4], a.timing_events[5] = ev[4], ev[5]
            self._phase(_lib.PHASE_INBATCH)
            a.timing_events[4] = a.timing_events[5] = None
            dp = yield ReduceScatter(self.ib_dp_all[: W * B])
            a.inbatch_dp = dp.data_ptr()
            ib = (gathered, dp)
        if self.cal:
            # ---- category alignment over the global batch: per-category sums, then scatters -------
            self._phase(_lib.PHASE_CAL_STATS)
            if W > 1:
                yield AllReduce(self.cal_stats)
            self._phase(_lib.PHASE_CAL_SCATTER)
            if W > 1:
                yield AllReduce(self.cal_scatter)
        # ---- scores; (dT | dA) to the owners; backward -------------------------------------------
        self._phase(_lib.PHASE_SCORE if self.group_towers else _lib.PHASE_USER)
        if W == 1:
            bwd_in = self.bwd_out[:R]
        else:
            self.exchange_floats[1] = bwd_src.numel()
            bwd_in = yield AllToAll(bwd_src, to_own, to_req)
        a.item_bwd_in = bwd_in.data_ptr()
        for i in (0, 1, 6, 7):  # table maintenance, wide weight-gradient GEMM
            a.timing_events[i] = ev[i]
        self._phase(_lib.PHASE_TOWERS_BWD if self.group_towers else _lib.PHASE_ITEM_BWD)
        for i in (6, 7):
            a.timing_events[i] = None
        if W > 1:
            yield AllReduce(self.arena)
        if self.clip:  # the table updates under the global clip coefficient
            self._phase(_lib.PHASE_TABLES)
        a.timing_events[0] = a.timing_events[1] = None
        self._phase(_lib.PHASE_DENSE)
        self.steps_done += 1
        self._register_sgd_buffers()
        # keep the step's device buffers alive until the stream has consumed them
        self._live = (route, back, bwd_in) + ib

    def _check_next_batch(self, users: torch.Tensor, pos: torch.Tensor) -> None:
        B = users.numel()
        if B == 0 or B > self.max_batch or users.dtype != torch.long or pos.dtype != torch.long or \
                pos.numel() != B:
            raise ValueError("ttamm: next_batch must be int64 (users, positives) of one size <= max_batch")
        if self.num_neg > 0 and self.csr is None:
            raise ValueError("ttamm: positives are required to sample negatives")

    def _look_ahead(self, users: torch.Tensor, pos: torch.Tensor) -> Program:
        """Program: the next step's id checks, negatives and request routing up to the count
        exchange (route_start with its host copy in flight).  Its status word starts as this
        rank's (an earlier poison rides along as in the step's own exchange).  The batch was
        validated before the step's first collective (_check_next_batch)."""
        W, rank = self.own.world_size, self.own.rank
        B, N = users.numel(), self.num_neg
        # cheap guards on the buffers the draws below write (the full check ran before the step's
        # first collective): never write past _ahead_bufs' max_batch x N slots
        if not (0 < B <= self.max_batch) or users.dtype != torch.long or pos.dtype != torch.long or \
                pos.numel() != B or (N > 0 and self.csr is None):
            raise RuntimeError("ttamm: look-ahead batch failed validation (internal error)")
        users0, pos0 = users, pos  # the next step's program finds its batch by identity
        users, pos = users.reshape(-1), pos.reshape(-1)
        dev = self.device
        if self._ahead_bufs is None:
            self._ahead_bufs = [torch.empty(self.max_batch * N, dtype=torch.long, device=dev) for _ in range(2)]
            self._ahead_status = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(2)]
            self._ahead_host = (torch.empty((2 * W, self.count_ld), dtype=torch.long, pin_memory=True)
                                if dev.type == "cuda" and W > 1 else None)
        k = self._ahead_flip
        self._ahead_flip ^= 1
        status = self._ahead_status[k]
        status.copy_(self.status)
        stream = _lib.stream_handle(dev)
        _lib.check(self.lib.ttamm_check_rows(users.data_ptr(), B, self.model.user_encoder.num_embeddings,
                                             pos.data_ptr(), B, self.num_items, status.data_ptr(), stream))
        negs = self._ahead_bufs[k][: B * N]
        base, Bg = rank * B, W * B
        if N > 0:
            _lib.check(self.lib.ttamm_sample_negatives(
                users.data_ptr(), B, N, self.num_items, self.csr.offsets.data_ptr(), self.csr.values.data_ptr(),
                self.csr.num_users, self.args.b.seed, self.steps_done + 1, base * N, negs.data_ptr(),
                status.data_ptr(), stream))
        pend = yield from route_start(self.own, self.router, pos, negs, base, Bg + base * N, status=status,
                                      host=self._ahead_host, ld=self.count_ld)
        return _Ahead(users0, pos0, negs, status, pend)

    def step(self, users, pos_items, neg_items=None, *, keep_masks=None, timing_events=None,
             next_batch=None) -> None:
        if self.comm is None:
            raise RuntimeError("ttamm: ShardedTrainStep.step needs comm= (e.g. TorchComm()); "
                               "use program() with run_loopback for in-process ranks")
        self.comm.run(self.program(users, pos_items, neg_items, keep_masks=keep_masks, timing_events=timing_events,
                                   next_batch=next_batch))

    def finish_program(self) -> Program:
        """Collective finish: global epoch loss (sum of the ranks' shares).  A status error on
        any rank (an out-of-range id, sampler exhaustion) raises on every rank, and every rank
        holds the state after the same last good step: the status words ride with each step's
        request counts, so a poisoned step is skipped by all ranks before any writes state."""
        self._ahead = None  # a look-ahead no step consumed: its exchange ran on every rank, nothing to undo
        bits = (_lib.STATUS_SAMPLER_EXHAUSTED, _lib.STATUS_INDEX_OUT_OF_RANGE, _lib.STATUS_LOOKAHEAD_MISMATCH)
        flags = torch.stack([(self.status & b) != 0 for b in bits]).reshape(-1).to(torch.float32)
        yield AllReduce(flags)
        for i, b in enumerate(bits):
            self.status.bitwise_or_((flags[i] > 0).to(torch.int32) * b)
        yield AllReduce(self.loss_accum)
        return FusedTrainStep.finish(self)

    def finish(self) -> float:
        if self.comm is None:
            raise RuntimeError("ttamm: ShardedTrainStep.finish needs comm=")
        return self.comm.run(self.finish_program())

    def last_losses(self) -> dict[str, float]:
        """Global losses of the last step (the all-reduced shares)."""
        return super().last_losses()


# ---------------------------------------------------------------------------------------
# the sharded epoch (training.py:1475-1490 over W ranks)
# ---------------------------------------------------------------------------------------
def route_pairs(own: RowOwnership, router: Router, users: torch.Tensor, items: torch.Tensor) -> Program:
    """Program: send every (user, item) pair to its user's owner (the all-to-all of SURVEY §8 e
    (a)).  Returns (local users, items, sizes): the pairs this rank owns — from rank 0, then
    rank 1, ..., each source's pairs in their order — and every rank's routed batch size.  The
    W x W count matrix is all-gathered once (one host sync) and gives the splits and sizes."""
    W = own.world_size
    packed, _, counts = router(W, users, None, items)
    if W == 1:
        return packed[:, 0].contiguous(), packed[:, 1].contiguous(), [users.numel()]
    m = yield AllGather(counts)
    m = m.reshape(W, W).tolist()  # m[src][dst]
    rank = own.rank
    got = yield AllToAll(packed, m[rank], [m[src][rank] for src in range(W)])
    sizes = [sum(m[src][dst] for src in range(W)) for dst in range(W)]
    return got[:, 0].contiguous(), got[:, 1].contiguous(), sizes


def epoch_program(engine: ShardedTrainStep, batches: Any) -> Program:
    """One epoch as an SPMD program: each rank iterates over its own part of the interaction
    stream (any users — e.g. a DeviceInteractionLoader over the rank's slice of the pairs, or a
    DistributedSampler); each batch's pairs are routed to their users' owners and the W routed
    batches form one global step (the reference step over their rank-major concatenation).
    Every rank must yield the same number of batches.  Returns the epoch's mean loss
    (training.py:829-833)."""
    own = engine.own
    rank = own.rank
    for users, items in batches:
        u, i, sizes = yield from route_pairs(own, engine.router, users, items)
        # every rank holds the same sizes (the all-gathered count matrix): they all raise here,
        # before the step's first collective, instead of one rank leaving the others waiting in it
        if min(sizes) == 0:
            raise ValueError("ttamm: a rank received no interactions for this step")
        if max(sizes) > engine.max_batch:
            raise ValueError(f"ttamm: a routed batch of {max(sizes)} interactions exceeds the sharded step's "
                             f"max_batch={engine.max_batch} (size it for the largest per-rank share of a step)")
        if engine.in_batch and len(set(sizes)) > 1:
            raise ValueError("ttamm: in-batch negatives need the same routed batch size on every rank "
                             f"(routed sizes {sizes}); feed each rank its own users' interactions instead")
        yield from engine.program(u, i, row_base=sum(sizes[:rank]), global_batch=sum(sizes))
    return (yield from engine.finish_program())


def train_one_epoch_sharded(engine: ShardedTrainStep, batches: Any, comm: Callable[[Program], Any] | None = None
                            ) -> float:
    """``train_one_epoch`` for one rank of a W-rank job: ``batches`` is this rank's part of the
    epoch's interactions; ``engine`` its ShardedTrainStep (sized with ``max_batch`` >= the largest
    routed batch).  Collective: every rank calls it with the same number of batches."""
    comm = comm or engine.comm
    if comm is None:
        raise RuntimeError("ttamm: train_one_epoch_sharded needs comm= (e.g. TorchComm())")
    runner = comm.run if hasattr(comm, "run") else comm
    return runner(epoch_program(engine, batches))
