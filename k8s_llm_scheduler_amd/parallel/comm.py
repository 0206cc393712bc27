"""Tensor-parallel process group: one process per GPU, collectives over RCCL (xGMI) or gloo (CPU tests).

On MI355X the backend string ``"nccl"`` IS RCCL.  The decode path issues 2 all-reduces per layer
(row-parallel O and down projections) plus one logits all-gather per step; all of them are
enqueued on the current HIP stream and are captured into the decode hipGraph.

Design choices for 8 x MI355X over point-to-point xGMI (7 links x ~153 GB/s per GPU):
* Decode messages are tiny (B x 8192 bf16 = 16 KiB at B = 1): latency-bound, so the collective
  is issued in-place on the producing tensor (no staging copies) and captured in the graph.
* The vocabulary-parallel LM head gathers fp32 logits [tp, B, V/tp] directly in shard-major
  order; the sampler consumes that layout without a transpose.
* Messages up to ``slot_bytes`` go through the native one-shot xGMI peer-memory collectives
  (``XgmiComm``, csrc/kernels/xgmi.hip): one fabric crossing instead of a ring's 2(W-1) hops.
  It is enabled only when every rank can map every peer's memory, it passes a self-test, and
  (``K8S_TP_COMM=auto``) it beats RCCL in a graph-timed probe on this node.  Larger messages
  (batched prefill) use RCCL.
"""

from __future__ import annotations

import datetime
import logging
import os
import pickle
import socket
import threading
import time
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.stages import stage


_DT = {torch.bfloat16: 0, torch.float32: 1, torch.float16: 2, torch.int32: 3}
log = logging.getLogger(__name__)


@dataclass
class TPGroup:
    rank: int = 0
    world: int = 1
    group: Optional[object] = None
    backend: str = "none"
    rccl: Optional[object] = None   # native RcclComm (GPU): graph-capturable collectives
    simulate: bool = False          # shapes of a TP rank, collectives skipped (profiling only)
    xgmi: Optional[object] = None   # native XgmiComm: one-shot peer-memory collectives (small messages)
    comm_info: dict = field(default_factory=dict)
    # Data parallelism over engine replicas (WORLD_SIZE = replicas x world): this rank is TP rank
    # ``rank`` of replica ``replica``, whose TP rank 0 is global rank ``leader``.
    replica: int = 0
    replicas: int = 1
    leader: int = 0

    @property
    def global_rank(self) -> int:
        return self.leader + self.rank

    xgmi_max_ar: int = 0            # all-reduces up to this size use xGMI (autotune_comm; 0 = capacity)

    # while a graph is being captured every all-reduce that fits the xGMI capacity runs on xGMI even where the
    # autotune found RCCL faster eagerly: a captured prefill chunk beats an eager one by far more than the
    # transport difference, and RCCL stays out of captured graphs (engine._prefill_bucket_capturable)
    capture_on_xgmi: bool = False
    rccl_calls: int = 0             # RCCL collectives issued from the host (a graph replay issues none)
    # transport of every all-reduce issued from the host, "<phase>:<transport>:<bytes>" -> calls (a captured graph's
    # all-reduces count once, at capture); ``phase`` is set by the model ("decode" / "prefill")
    phase: str = "eager"
    ar_log: dict = field(default_factory=dict)

    def _log_ar(self, transport: str, nbytes: int) -> None:
        k = f"{self.phase}:{transport}:{nbytes}"
        self.ar_log[k] = self.ar_log.get(k, 0) + 1

    def _xgmi_ok(self, t: torch.Tensor, reduce: bool = False) -> bool:
        n = t.numel() * t.element_size()
        if self.xgmi is None or not t.is_cuda or n % 16 or n <= 0:
            return False
        if reduce:
            cap = self.xgmi.max_allreduce_bytes
            return n <= (cap if self.capture_on_xgmi else (self.xgmi_max_ar or cap))
        return n <= self.xgmi.slot_bytes

    @property
    def enabled(self) -> bool:
        return self.world > 1

    def all_reduce_(self, t: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """In-place sum over the TP group; with ``residual`` the result is sum + residual (the xGMI
        kernels fuse the residual add, SURVEY K14 + K2; other transports add it afterwards)."""
        if self.world > 1 and not self.simulate:
            nbytes = t.numel() * t.element_size()
            if t.dtype == torch.bfloat16 and t.is_contiguous() and self._xgmi_ok(t, reduce=True):
                self._log_ar("xgmi", nbytes)
                rp = 0
                if residual is not None:
                    if residual.dtype != t.dtype or residual.shape != t.shape or not residual.is_contiguous():
                        raise ValueError("residual must match the reduced tensor")
                    rp = residual.data_ptr()
                self.xgmi.all_reduce_bf16(t.data_ptr(), t.data_ptr(), t.numel() * 2, -1, rp)
                return t
            elif self.rccl is not None and t.is_cuda:
                self._log_ar("rccl", nbytes)
                self.rccl_calls += 1
                self.rccl.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], 0, -1)
            elif self.backend == "gloo" and t.dtype == torch.bfloat16:
                self._log_ar("gloo", nbytes)
                f = t.float()
                dist.all_reduce(f, group=self.group)
                t.copy_(f)
            else:
                dist.all_reduce(t, group=self.group)
            if residual is not None:
                t.add_(residual)
        return t

    fused_ar: bool = os.environ.get("K8S_FUSED_AR", "1") != "0"

    def linear_all_reduce(self, x: torch.Tensor, w, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``residual + all_reduce(x @ w.T)`` for a row-parallel projection (o_proj / down).  Decode rows on the
        xGMI transport run ONE kernel: the GEMV pushes its partial rows to every peer in its epilogue and reduces
        them there (kernels/gemv.hip GemvAr; ``K8S_FUSED_AR=0`` restores GEMV + separate all-reduce kernel).  The
        result has the bits of the separate path."""
        from .. import ops

        if (self.fused_ar and self.world > 1 and not self.simulate and self.xgmi is not None and x.is_cuda
                and x.dim() == 2 and x.shape[0] <= ops.GEMV_MAX_M and (residual is None or residual.is_contiguous())):
            y = ops.gemv_allreduce(self.xgmi, x, w, residual)
            if y is not None:
                self._log_ar("fused_gemv_ar", y.numel() * y.element_size())
                return y
        y = ops.linear(x, w)
        return self.all_reduce_(y, residual=residual)

    def all_gather_shards(self, t: torch.Tensor) -> torch.Tensor:
        """[..] local -> [world, ..] (shard-major)."""
        if self.world == 1:
            return t.unsqueeze(0)
        if self.simulate:
            return t.unsqueeze(0).expand(self.world, *t.shape).contiguous()
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        t = t.contiguous()
        if self._xgmi_ok(t):
            self.xgmi.all_gather(t.data_ptr(), out.data_ptr(), t.numel() * t.element_size(), -1)
        elif self.rccl is not None and t.is_cuda:
            self.rccl_calls += 1
            self.rccl.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), _DT[t.dtype], -1)
        elif self.backend == "gloo":
            dist.all_gather(list(out.unbind(0)), t.contiguous(), group=self.group)
        else:
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    def reduce_scatter_rows(self, t: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sequence parallelism (SURVEY 2.6 P-SP): rows [rank * n, (rank + 1) * n) of the sum over the TP group of
        ``t`` [world * n, ...], plus ``residual`` (this rank's n rows of the residual stream).  RCCL reduce-scatter
        where a communicator exists; otherwise the all-reduce transports (xGMI, gloo) and this rank's rows -- the
        same sum.  ``t`` may be overwritten."""
        T = t.shape[0]
        if T % self.world:
            raise ValueError(f"reduce_scatter_rows: {T} rows do not split over {self.world} ranks")
        n = T // self.world
        if self.world == 1:
            out = t
        elif self.simulate:
            out = t[:n]                    # one rank's shapes, collective skipped
        elif self.rccl is not None and t.is_cuda and t.dtype in _DT:
            t = t.contiguous()
            out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            self.rccl_calls += 1
            self.rccl.reduce_scatter(t.data_ptr(), out.data_ptr(), out.numel(), _DT[t.dtype], 0, -1)
        else:
            out = self.all_reduce_(t.contiguous())[self.rank * n:(self.rank + 1) * n]
        if residual is not None:
            out.add_(residual)
        return out

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """[n, ...] row shard of every rank -> [world * n, ...] in rank order (the inverse of reduce_scatter_rows)."""
        if self.world == 1:
            return t
        g = self.all_gather_shards(t)
        return g.view((g.shape[0] * g.shape[1],) + tuple(g.shape[2:]))

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world > 1:
            dist.broadcast(t, src=self.leader + src, group=self.group)
        return t

    def barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.group)

    # ---- failure detection (engine faults must reach the retry / breaker path)
    failed: Optional[str] = None    # sticky: set by check_health on the first collective failure

    def ensure_healthy(self) -> None:
        """Fail fast (before launching more collectives) once a failure has been seen."""
        if self.failed:
            raise CollectiveError(self.failed)

    def snapshot_health(self) -> None:
        """Enqueue (on the current stream) a copy of the xGMI error word to pinned host memory; read
        by :meth:`check_health` after the caller's own stream synchronisation (no extra sync)."""
        if self.xgmi is not None and not self.simulate:
            self.xgmi.snapshot_error(-1)

    def check_health(self) -> None:
        """Raise :class:`CollectiveError` if a collective failed since the communicator was built: an
        xGMI poll timed out (a peer stalled or died; the kernel drained with partial sums) or RCCL
        reports an asynchronous error.  The error is sticky -- the ranks' collective sequences are
        out of step, so every later call fails fast until the engine is rebuilt."""
        if self.simulate or self.world <= 1:
            return
        self.ensure_healthy()
        if self.xgmi is not None:
            mask = int(self.xgmi.last_error())
            if mask:
                self.failed = (f"xGMI collective timed out waiting for peer rank(s) "
                               f"{[r for r in range(self.world) if mask >> r & 1]} (rank {self.rank})")
        if self.rccl is not None and not self.failed:
            err = self.rccl.async_error()
            if err:
                self.failed = f"RCCL communicator error on rank {self.rank}: {err}"
        self.ensure_healthy()


    def reset_collectives(self, control: Optional["ControlChannel"] = None, timeout_s: float = 60.0) -> None:
        """Recovery after a collective failure or stall (every rank of the replica calls this, with its device
        drained): the xGMI protocol state goes back to its freshly-built state on every rank, an aborted or
        failed RCCL communicator is replaced by a new one (unique id from the leader over the gloo control
        group), and a bounded barrier makes sure no rank issues a collective before every rank has reset."""
        if self.world <= 1 or self.simulate:
            self.failed = None
            return
        if (self.xgmi is not None or self.rccl is not None) and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        if self.xgmi is not None:
            self.xgmi.reset()
        rebuild = self.rccl is not None and bool(self.rccl.aborted or self.rccl.async_error())
        if control is not None:
            # one decision for the whole replica: a rank whose own communicator looks healthy (it never saw the
            # stall) must still take part in the rebuild the others need, or the collectives below do not match
            control.barrier(timeout_s)
            rebuild = control.any_rank(rebuild, timeout_s)
        if rebuild:
            from .. import ops

            if control is None:
                raise CollectiveError("RCCL communicator rebuild needs the control channel")
            if not self.rccl.aborted:
                self.rccl.abort()
            uid = ops.native().RcclComm.unique_id() if self.rank == 0 else None
            uid = control.broadcast_object(uid)
            self.rccl = ops.native().RcclComm(self.world, self.rank, uid)
        if control is not None:
            control.barrier(timeout_s)
        self.failed = None

    def abort_rccl(self) -> None:
        """Abort the RCCL communicator so operations parked on a dead peer error out and the stream drains."""
        if self.rccl is not None and not self.rccl.aborted:
            self.rccl.abort()
            self.failed = self.failed or f"RCCL communicator aborted on rank {self.rank}"


class CollectiveError(RuntimeError):
    """A tensor-parallel collective failed; the decode results of this step are not trustworthy."""


class ControlChannel:
    """TP-rank-0 -> replica schedule messages on a CPU (gloo) group: the replica's leader (global rank 0
    runs the serving control plane) announces new requests, aborts, reset commands and mid-chunk decisions,
    every other TP rank follows its engine schedule (engine.LLMEngine._sync).  The messages are one-way and
    posted asynchronously (isend), so a follower that stalls never blocks the leader's host loop (the leader's
    bounded device waits catch the stall).

    Followers report failures the other way through the process group's TCP store (``report_failure``);
    the leader polls it from a background thread (``peer_failure``), so a collective failure seen by ONE
    rank -- a peer that timed out waiting for a stalled leader -- reaches the leader without a per-step
    round trip."""

    def __init__(self, rank: int, group=None, src: int = 0, replica: int = 0, world: int = 1):
        self.rank = rank      # TP rank within the replica
        self.group = group
        self.src = src        # global rank of the replica's leader
        self.replica = replica
        self.world = world
        self._store = None
        self._failure: Optional[str] = None
        self._monitor: Optional[threading.Thread] = None
        self._monitor_stop = threading.Event()

    # Leader -> follower traffic is point-to-point and ASYNCHRONOUS on the leader (gloo isend; a broadcast would
    # wait for every follower to post its receive, so one stalled follower would stall the leader's host loop).
    # Followers receive in order (blocking: they only follow).  Tags: 1 schedule length, 2 schedule bytes,
    # 3 decisions.
    def _post(self, t: torch.Tensor, tag: int) -> None:
        pend = [(w, b) for w, b in getattr(self, "_pending", []) if not w.is_completed()]
        for dst in range(self.src + 1, self.src + self.world):
            pend.append((dist.isend(t, dst=dst, group=self.group, tag=tag), t))
        self._pending = pend   # keeps each sent tensor alive until its send completed

    def exchange(self, payload):
        """Leader: post ``payload`` (any picklable schedule message) to every follower and return it.  Follower:
        the leader's next message."""
        if self.world <= 1:
            return payload
        if self.rank == 0:
            data = pickle.dumps(payload)
            self._post(torch.tensor([len(data)], dtype=torch.int64), 1)
            self._post(torch.frombuffer(bytearray(data), dtype=torch.uint8), 2)
            return payload
        hdr = torch.zeros(1, dtype=torch.int64)
        dist.recv(hdr, src=self.src, group=self.group, tag=1)
        buf = torch.empty(int(hdr[0]), dtype=torch.uint8)
        dist.recv(buf, src=self.src, group=self.group, tag=2)
        return pickle.loads(buf.numpy().tobytes())

    def flush(self, timeout_s: float = 30.0) -> None:
        """Leader: wait (bounded) for the posted messages to be delivered (before the process group goes away)."""
        end = time.monotonic() + timeout_s
        for w, _ in getattr(self, "_pending", []):
            while not w.is_completed() and time.monotonic() < end:
                time.sleep(1e-3)
        self._pending = []

    # ---- failure reports (followers -> leader)
    def _key(self, rank: int) -> str:
        return f"k8s_engine_failure/{self.replica}/{rank}"

    def store(self):
        if self._store is None:
            try:
                self._store = dist.distributed_c10d._get_default_store()
            except Exception:  # noqa: BLE001 -- no store (single process): reports are dropped
                self._store = False
        return self._store or None

    def report_failure(self, reason: str) -> None:
        st = self.store()
        if st is not None:
            st.set(self._key(self.rank), reason[:500])

    def clear_failures(self) -> None:
        st = self.store()
        if st is not None:
            for r in range(self.world):
                st.set(self._key(r), "")
        self._failure = None

    def start_monitor(self, period_s: float = 0.05) -> None:
        """Leader: poll the followers' failure keys in the background."""
        if self.rank != 0 or self.world <= 1 or self._monitor is not None or self.store() is None:
            return
        keys = [self._key(r) for r in range(1, self.world)]

        def run():
            st = self.store()
            while not self._monitor_stop.is_set() and dist.is_initialized():
                try:
                    for k in keys:
                        if st.check([k]):
                            v = st.get(k).decode()
                            if v and self._failure is None:
                                self._failure = f"TP rank {k.rsplit('/', 1)[1]} failed: {v}"
                except Exception:  # noqa: BLE001 -- store gone (shutdown)
                    return
                self._monitor_stop.wait(period_s)

        self._monitor = threading.Thread(target=run, name="tp-health-monitor", daemon=True)
        self._monitor.start()

    def peer_failure(self) -> Optional[str]:
        return self._failure

    def stop_monitor(self) -> None:
        """Before the process group goes away (the monitor thread uses its store)."""
        self._monitor_stop.set()
        if self._monitor is not None:
            self._monitor.join(timeout=5)
            self._monitor = None

    def barrier(self, timeout_s: float) -> None:
        """Bounded barrier of the replica (gloo monitored barrier: raises if a rank does not arrive)."""
        dist.monitored_barrier(group=self.group, timeout=datetime.timedelta(seconds=timeout_s))

    def _reset_key(self) -> str:
        return f"k8s_engine_reset/{self.replica}"

    def request_reset(self) -> None:
        """Leader: bump the replica's reset generation (followers parked in a device wait poll it)."""
        st = self.store()
        if st is not None:
            st.add(self._reset_key(), 1)

    def reset_generation(self) -> int:
        st = self.store()
        if st is None:
            return 0
        return int(st.add(self._reset_key(), 0))

    def decide(self, value: int) -> int:
        """The leader's small integer decision (e.g. end a decode chunk early) to every rank of the replica: one
        int64 posted to each follower; followers pass anything and get the leader's value."""
        if self.world <= 1:
            return value
        if self.rank == 0:
            self._post(torch.tensor([value], dtype=torch.int64), 3)
            return value
        buf = torch.zeros(1, dtype=torch.int64)
        dist.recv(buf, src=self.src, group=self.group, tag=3)
        return int(buf[0])

    _vote_gen = -1
    _votes = 0

    def _vote_round(self) -> str:
        """Id of the next bounded vote, the same on every rank: the replica's reset generation (shared through the
        store; the leader bumps it before every announced reset) and the vote's index within it.  A rank whose vote
        of one generation failed cannot shift the others' rounds for good: the next generation starts at 0."""
        gen = self.reset_generation()
        if gen != self._vote_gen:
            self._vote_gen, self._votes = gen, 0
        self._votes += 1
        return f"{gen}.{self._votes}"

    def any_rank(self, flag: bool, timeout_s: Optional[float] = None) -> bool:
        """True on every rank of the replica iff ``flag`` is true on any of them (every rank must call this).
        ``timeout_s``: a bounded vote through the process group's TCP store (each rank sets its key, then waits
        for every rank's key at most that long and raises :class:`CollectiveError` otherwise) -- a rank that dies
        between the recovery barrier and this vote cannot park the others for the group's default timeout.  The
        last rank to finish reading deletes the round's keys (the store does not grow with every recovery)."""
        if self.world <= 1:
            return bool(flag)
        st = self.store() if timeout_s is not None else None
        if st is None:
            flags = [None] * self.world
            dist.all_gather_object(flags, bool(flag), group=self.group)
            return any(flags)
        rnd = self._vote_round()
        keys = [f"k8s_vote/{self.replica}/{rnd}/{r}" for r in range(self.world)]
        st.set(keys[self.rank], "1" if flag else "0")
        try:
            st.wait(keys, datetime.timedelta(seconds=timeout_s))
        except Exception as e:  # noqa: BLE001 -- store timeout / store gone
            raise CollectiveError(f"recovery vote timed out after {timeout_s:.0f}s on rank {self.rank}: {e}") from e
        out = any(st.get(k) == b"1" for k in keys)
        done = f"k8s_vote_done/{self.replica}/{rnd}"
        if st.add(done, 1) == self.world:      # every rank has read every key
            for k in keys + [done]:
                try:
                    st.delete_key(k)
                except Exception:  # noqa: BLE001 -- a store without delete: the keys stay (harmless)
                    pass
        return out

    def broadcast_object(self, obj):
        box = [obj]
        dist.broadcast_object_list(box, src=self.src, group=self.group)
        return box[0]


def replica_ranks(tp: TPGroup, replica: int) -> list:
    return list(range(replica * tp.world, (replica + 1) * tp.world))


def make_control_channel(tp: TPGroup) -> Optional[ControlChannel]:
    """Every rank must call this (torch.distributed.new_group is collective over the world)."""
    if tp.world <= 1 or tp.simulate:
        return None
    mine = None
    for r in range(tp.replicas):
        ranks = replica_ranks(tp, r) if tp.replicas > 1 else None
        g = dist.new_group(ranks=ranks, backend="gloo", timeout=datetime.timedelta(days=7))
        if r == tp.replica:
            mine = g
    return ControlChannel(tp.rank, mine, src=tp.leader, replica=tp.replica, world=tp.world)


def init_from_env(device_type: Optional[str] = None, timeout_s: int = 600, backend: Optional[str] = None,
                  comm: Optional[str] = None, tp_size: int = 0) -> TPGroup:
    """Initialise torch.distributed from torchrun env (RANK/WORLD_SIZE/MASTER_*).  Single
    process when WORLD_SIZE is unset or 1.

    ``tp_size`` (env ``K8S_TP``; 0 = WORLD_SIZE): tensor-parallel degree of one engine replica.
    WORLD_SIZE / tp_size replicas of ranks [r*tp, (r+1)*tp) each hold a full model copy (data
    parallelism over decisions, e.g. two TP=4 half-node engines on 8 GPUs); each replica gets its
    own process group, RCCL communicator and xGMI peer regions.

    ``backend``: process-group backend (default ``nccl`` = RCCL on GPU, ``gloo`` on CPU; env
    ``K8S_TP_BACKEND``).  ``comm`` (env ``K8S_TP_COMM``): ``auto`` = RCCL plus the xGMI one-shot
    collectives when they are faster, ``rccl`` = RCCL only, ``xgmi`` = xGMI for every message that
    fits (no RCCL communicator at all under a gloo process group, e.g. several ranks sharing one GPU
    in tests).  Rank r uses GPU ``LOCAL_RANK % device_count``."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world <= 1:
        return TPGroup()
    tp_size = int(tp_size or os.environ.get("K8S_TP", "0") or 0) or world
    if tp_size < 1 or world % tp_size:
        raise ValueError(f"WORLD_SIZE {world} is not a multiple of the TP degree {tp_size}")
    replicas = world // tp_size
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    backend = backend or os.environ.get("K8S_TP_BACKEND")
    comm = comm or os.environ.get("K8S_TP_COMM")
    if backend is None and device_type == "cuda" and torch.cuda.device_count() < min(world, tp_size):
        # more ranks than GPUs (ranks sharing a GPU: the one-GPU rehearsal of a node): RCCL refuses two ranks on one
        # device, so the process group is gloo and the collectives are the xGMI peer-memory kernels alone
        backend, comm = "gloo", comm or "xgmi"
        log.warning(f" {world} ranks on {torch.cuda.device_count()} GPU(s): gloo process group, xGMI collectives")
    backend = backend or ("nccl" if device_type == "cuda" else "gloo")
    comm = comm or "auto"
    if comm not in ("auto", "rccl", "xgmi"):
        raise ValueError(f"K8S_TP_COMM must be auto, rccl or xgmi (got {comm!r})")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        kw = {}
        if device_type == "cuda":
            local = int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            if backend == "nccl":
                kw["device_id"] = torch.device("cuda", local)
        with stage("process_group"):
            dist.init_process_group(backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
    replica = rank // tp_size
    group = dist.group.WORLD
    if replicas > 1:   # collective: every rank creates every replica's group, in order
        for r in range(replicas):
            g = dist.new_group(ranks=list(range(r * tp_size, (r + 1) * tp_size)))
            if r == replica:
                group = g
    tp = TPGroup(rank % tp_size, tp_size, group, backend, replica=replica, replicas=replicas,
                 leader=replica * tp_size)
    if tp_size == 1:
        return tp   # pure data parallelism: no collectives inside the model
    if device_type == "cuda":
        if backend == "nccl" and comm in ("auto", "rccl"):
            with stage("rccl_init"):
                tp.rccl = make_rccl_comm(tp)
        if comm in ("auto", "xgmi"):
            tp.xgmi = make_xgmi_comm(tp)
        tune = os.environ.get("K8S_COMM_AUTOTUNE", "1")
        # ranks time-sharing one GPU (the 1-GPU rehearsals) measure the scheduler, not the transports:
        # keep the built-in thresholds there unless forced
        own_gpu = torch.cuda.device_count() >= tp_size
        if tp.xgmi is not None and (tune == "force" or (tune == "1" and own_gpu)):
            with stage("comm_autotune"):
                autotune_comm(tp)   # thresholds between the xGMI protocols (and RCCL, when present)
        tp.comm_info["selected"] = "xgmi+rccl" if tp.xgmi is not None and tp.rccl is not None else \
            ("xgmi" if tp.xgmi is not None else ("rccl" if tp.rccl is not None else backend))
    return tp


def make_rccl_comm(tp: TPGroup):
    """Create the engine's own RCCL communicator (unique id broadcast over torch.distributed)."""
    from .. import ops

    _C = ops.native()
    dev = torch.device("cuda", torch.cuda.current_device())
    uid = torch.zeros(128, dtype=torch.uint8, device=dev)
    if tp.rank == 0:
        uid.copy_(torch.frombuffer(bytearray(_C.RcclComm.unique_id()), dtype=torch.uint8))
    dist.broadcast(uid, src=tp.leader, group=tp.group)
    comm = _C.RcclComm(tp.world, tp.rank, bytes(uid.cpu().tolist()))
    # one eager collective so lazy RCCL setup happens outside any graph capture
    probe = torch.ones(16, dtype=torch.float32, device=dev)
    comm.all_reduce(probe.data_ptr(), probe.data_ptr(), probe.numel(), 1, 0, -1)
    torch.cuda.synchronize(dev)
    if float(probe[0]) != float(tp.world):
        raise RuntimeError(f"RCCL communicator self-test failed: {float(probe[0])} != {tp.world}")
    return comm


def _agree(tp: TPGroup, ok: bool) -> bool:
    """True iff ``ok`` on every rank (every rank must call this)."""
    flags = [None] * tp.world
    dist.all_gather_object(flags, bool(ok), group=tp.group)
    return all(flags)


XGMI_AR_CAPACITY = 8 << 20   # the largest all-reduce on the xGMI transports: a 512-token chunk of 70B (8192 x bf16)


def default_slot_bytes(world: int) -> int:
    """Per-peer slot of the xGMI region: every all-reduce up to XGMI_AR_CAPACITY fits (two-shot capacity is world x
    slot), so a decision's prefill chunk (<= 512 tokens, 8 MiB per all-reduce at 70B) stays on the graph-capturable
    peer-memory path at every TP degree; at least 4 MiB, so the decode step's logits all-gather (rows x vocab / TP
    fp32 per rank: 4.1 MB at TP=8 and 64 rows) stays on xGMI inside the decode graphs too.  The region holds
    10 x world slots: 80-320 MiB of the 288 GB."""
    return max(4 << 20, (XGMI_AR_CAPACITY // max(1, world) + 4095) // 4096 * 4096)


def make_xgmi_comm(tp: TPGroup, slot_bytes: Optional[int] = None, blocks: Optional[int] = None,
                   timeout_s: float = 60.0):
    """Map every rank's IPC region into every process and self-test the one-shot collectives.
    Returns None (on every rank alike) when any rank cannot take part."""
    from .. import ops

    slot_bytes = int(slot_bytes or os.environ.get("K8S_XGMI_MAX_BYTES", 0) or default_slot_bytes(tp.world))
    slot_bytes = (slot_bytes + 4095) // 4096 * 4096
    blocks = int(blocks or os.environ.get("K8S_XGMI_BLOCKS", 16))
    timeout_s = float(os.environ.get("K8S_XGMI_TIMEOUT_S", timeout_s))
    dev = torch.cuda.current_device()
    comm, handle, err = None, b"", ""
    try:
        if tp.world > 8:
            raise RuntimeError("more than 8 ranks")
        comm = ops.native().XgmiComm(tp.world, tp.rank, slot_bytes, blocks, timeout_s)
        comm.ll_max_bytes = int(os.environ.get("K8S_XGMI_LL_MAX", 64 * 1024))
        handle = comm.handle()
    except Exception as e:  # noqa: BLE001 -- every rank must still join the exchange below
        err = str(e)
    info = [None] * tp.world
    dist.all_gather_object(info, (socket.gethostname(), dev, handle, err), group=tp.group)
    ok = all(h == info[0][0] and hd and not er for h, _, hd, er in info)
    with stage("xgmi_open"):
        if ok:
            try:
                for _, d, _, _ in info:
                    if d != dev and not torch.cuda.can_device_access_peer(dev, d):
                        raise RuntimeError(f"GPU {dev} cannot access GPU {d}")
                comm.open([x[2] for x in info])
            except Exception as e:  # noqa: BLE001
                ok, err = False, str(e)
        ok = _agree(tp, ok)
    if not ok:
        reasons = sorted({x[3] for x in info if x[3]} | ({err} if err else set()))
        why = '; '.join(reasons) or 'a peer could not map memory'
        tp.comm_info["xgmi"] = f"disabled: {why}"
        log.warning(f" xGMI peer-memory collectives disabled: {why}")
        return None
    with stage("xgmi_selftest"):
        ok = _agree(tp, _xgmi_selftest(tp, comm, dev))
    if not ok:
        tp.comm_info["xgmi"] = "disabled: self-test failed"
        log.warning(" xGMI peer-memory collectives disabled: self-test failed")
        return None
    tp.comm_info["xgmi"] = "self-test passed"
    # the GEMV with the all-reduce in its epilogue (decode O / down projections): bit-exact against GEMV + the LL
    # all-reduce on this node's links, or the decode falls back to the separate kernels (same bits, one launch more)
    with stage("fused_ar_selftest"):
        fused_ok = _agree(tp, _fused_ar_selftest(tp, comm, dev))
    tp.comm_info["fused_gemv_ar_selftest"] = "passed" if fused_ok else "failed"
    if not fused_ok:
        log.warning(" fused GEMV all-reduce disabled: self-test failed (decode uses GEMV + xGMI all-reduce)")
        tp.fused_ar = False
        # a failed check may have timed out in a poll: clear the sticky error word and the protocol state on every
        # rank (after every rank has drained: _agree above), or the engine's first health check reports that stale
        # timeout as a collective failure of its own
        comm.reset()
        _agree(tp, True)
    return comm


def _xgmi_selftest(tp: TPGroup, comm, dev) -> bool:
    try:
        sizes = [min(comm.slot_bytes // 2, 64 * 1024)]               # flagged one-shot path
        if comm.ll_max_bytes >= 2:
            sizes.append(min(comm.ll_max_bytes, comm.slot_bytes // 2) // 2)  # LL path (flag in every word)
        for it in range(3 * len(sizes)):  # both slots, then the first again, for every path
            n = sizes[it % len(sizes)]
            x = (torch.arange(n, device=dev, dtype=torch.float32) % 61 + tp.rank * 3 + it).to(torch.bfloat16)
            want = sum((torch.arange(n, device=dev, dtype=torch.float32) % 61 + r * 3 + it) for r in range(tp.world))
            comm.all_reduce_bf16(x.data_ptr(), x.data_ptr(), n * 2, -1)
            g_in = torch.full((1024,), float(tp.rank + it), device=dev)
            g_out = torch.empty((tp.world, 1024), device=dev)
            comm.all_gather(g_in.data_ptr(), g_out.data_ptr(), 4096, -1)
            torch.cuda.synchronize(dev)
            if comm.error() != 0:
                return False
            if not torch.equal(x.float(), want.to(torch.bfloat16).float()):
                return False
            if not torch.equal(g_out[:, 0].cpu(), torch.arange(tp.world, dtype=torch.float32) + it):
                return False
        return True
    except Exception as e:  # noqa: BLE001
        log.warning(f" xGMI self-test raised: {e}")
        return False


def fused_ar_selftest_shapes(world: int) -> list:
    """(M, N, K) of the fused GEMV all-reduce start-up check beyond 1 x 1024 x 1024: the decode row-parallel shards of
    Llama-3.3-70B at this TP degree (O: K = 8192 / tp, down: K = 28672 / tp; N = hidden 8192), at 1 and 2 rows."""
    out = []
    for k in (8192, 28672):
        if k % world == 0:
            out += [(m, 8192, k // world) for m in (1, 2)]
    return out


def _fused_ar_oracle_check(tp: TPGroup, comm, dev, shapes) -> bool:
    """gemv_allreduce at ``shapes`` against the fp32 oracle sum over ranks of x_r @ W_r^T + residual (every rank
    regenerates every rank's operands from a per-rank seed on the device), within bf16 rounding."""
    from .. import ops

    for i, (M, N, K) in enumerate(shapes):
        def operands(r):
            g = torch.Generator(device=dev).manual_seed(7919 * (i + 1) + r)
            x = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, generator=g, device=dev) * (0.5 / K ** 0.5)).to(torch.bfloat16)
            return x, w
        g = torch.Generator(device=dev).manual_seed(104729 + i)
        res = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16)
        x, w = operands(tp.rank)
        for _ in range(2):   # both epoch parities
            y = ops.gemv_allreduce(comm, x, w, res)
            if y is None:
                log.warning(f" fused GEMV all-reduce refused the 70B shard shape {(M, N, K)}")
                return False
            want = res.float()
            for r in range(tp.world):
                xr, wr = operands(r)
                want = want + xr.float() @ wr.float().T
            torch.cuda.synchronize(dev)
            err = float((y.float() - want).abs().max())
            ew = comm.error()
            if ew != 0 or not err <= 0.02 * float(want.abs().max()) + 0.05:
                log.warning(f" fused GEMV all-reduce {(M, N, K)}: max |error| {err:.4g} vs the fp32 oracle, error word "
                            f"{ew:#x} (rank {tp.rank})")
                return False
            del want
    return True


def _fused_ar_selftest(tp: TPGroup, comm, dev) -> bool:
    """gemv.hip GemvAr over the mapped peer regions vs GEMV + the LL all-reduce (+ residual), bitwise, twice (both
    epoch parities); the 70B decode shard shapes (fused_ar_selftest_shapes) against the fp32 oracle; the two-shot
    kernel at 1 MiB against the fixed-order fp32 sum."""
    from .. import ops

    try:
        M, N, K = 1, 1024, 1024
        g = torch.Generator().manual_seed(17)
        xs = [torch.randn(M, K, generator=g).to(torch.bfloat16) for _ in range(tp.world)]
        ws = [(torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16) for _ in range(tp.world)]
        r = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
        x, w = xs[tp.rank].to(dev), ws[tp.rank].to(dev)
        keep = comm.ll_max_bytes
        comm.ll_max_bytes = max(keep, 2 * M * N)
        try:
            for _ in range(2):
                y = ops.gemv_allreduce(comm, x, w, r)
                if y is None:
                    return True            # shape outside the fused plan: nothing to check, nothing used
                base = ops.linear(x, w)
                comm.all_reduce_bf16(base.data_ptr(), base.data_ptr(), M * N * 2, -1, r.data_ptr())
                torch.cuda.synchronize(dev)
                if comm.error() != 0 or not torch.equal(y, base):
                    return False
            # (8 processes TIME-SHARING one GPU -- the rehearsals -- stall the 1024-workgroup 70B-shape launches in
            # their peer polls at random, whatever the shape: profiles/fused_ar_70b_shapes_r6.txt; the same shapes pass
            # with 2 and 4 processes per GPU.  Beyond 4 the check is skipped; ranks with a GPU each always run it)
            per_gpu = -(-dist.get_world_size() // max(1, torch.cuda.device_count()))   # processes sharing a GPU
            if per_gpu <= 4 and not _fused_ar_oracle_check(tp, comm, dev, fused_ar_selftest_shapes(tp.world)):
                return False
        finally:
            comm.ll_max_bytes = keep
        n = (1 << 20) // 2
        if 2 * n <= comm.max_allreduce_bytes:
            keep2 = comm.twoshot_min_bytes
            comm.twoshot_min_bytes = 16
            try:
                parts = [(torch.arange(n, dtype=torch.float32) % 97 - 48 + 5 * q).to(torch.bfloat16)
                         for q in range(tp.world)]
                t = parts[tp.rank].to(dev)
                comm.all_reduce_bf16(t.data_ptr(), t.data_ptr(), 2 * n, -1)
                torch.cuda.synchronize(dev)
                want = sum(p.float() for p in parts).to(torch.bfloat16)
                if comm.error() != 0 or not torch.equal(t.cpu(), want):
                    return False
            finally:
                comm.twoshot_min_bytes = keep2
        return True
    except Exception as e:  # noqa: BLE001
        log.warning(f" fused GEMV all-reduce self-test raised: {e}")
        return False


def _graph_time_us(fn, iters: int = 32, reps: int = 5) -> float:
    """Per-call time of ``fn`` (a collective) captured ``iters`` times into one hipGraph."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters * 1e6)
    return best


def comm_thresholds(table: dict, cap: int):
    """Transport thresholds from graph-timed all-reduces, ``table`` = {bytes: {"ll"?, "oneshot"?, "twoshot", "rccl"?:
    us}} (max over ranks): (LL up to the largest size where it is no slower than both one-shot kernels, two-shot from
    the smallest size where it beats the flagged one-shot, xGMI up to the largest size where its best kernel beats
    RCCL -- the whole xGMI capacity ``cap`` if it wins at the largest size measured)."""
    ll_max = max([n for n, r in table.items() if "ll" in r and r["ll"] <= min(r.get("oneshot", 1e9), r["twoshot"])],
                 default=0)
    two_min = min([n for n, r in table.items() if r["twoshot"] < r.get("oneshot", 1e9)], default=0)
    best = {n: min(v for k, v in r.items() if k != "rccl") for n, r in table.items()}
    xgmi_max = max([n for n in table if "rccl" not in table[n] or best[n] < table[n]["rccl"]], default=0)
    if table and xgmi_max == max(table):
        xgmi_max = cap
    return ll_max, two_min, xgmi_max


def autotune_comm(tp: TPGroup, sizes=(16384, 65536, 262144, 1 << 20, 4 << 20, 8 << 20)) -> None:
    """Graph-time every all-reduce transport at every message size class the engine issues (decode B=1:
    16 KiB; batched decode: up to 1 MiB at B=64; prefill chunks: MiBs), max over ranks, and set the
    thresholds: the LL protocol up to the largest size it wins, the two-shot kernel from the smallest
    size it beats the one-shot kernel, and xGMI at all only up to the largest size where it beats RCCL.
    Results land in ``tp.comm_info`` (bench.py reports them)."""
    dev = torch.cuda.current_device()
    xg, rc = tp.xgmi, tp.rccl
    cap = xg.max_allreduce_bytes
    sizes = [n for n in sizes if n <= cap]
    buf = torch.ones(max(sizes) // 2, dtype=torch.bfloat16, device=dev)
    keep = (xg.ll_max_bytes, xg.twoshot_min_bytes)
    table = {}

    def timed(fn) -> float:
        dist.barrier(group=tp.group)
        us = _graph_time_us(fn)
        t = torch.tensor([us], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=tp.group)
        return float(t[0])

    for n in sizes:
        row = {}
        variants = []
        if 2 * n <= xg.slot_bytes:
            variants.append(("ll", n + 1, 0))              # LL for this size
        if n <= xg.slot_bytes:
            variants.append(("oneshot", 0, 0))             # flagged one-shot
        variants.append(("twoshot", 0, 16))                # two-shot for everything
        for name, ll, two in variants:
            xg.ll_max_bytes, xg.twoshot_min_bytes = ll, two
            row[name] = round(timed(lambda: xg.all_reduce_bf16(buf.data_ptr(), buf.data_ptr(), n, -1)), 2)
        if rc is not None:
            row["rccl"] = round(timed(lambda: rc.all_reduce(buf.data_ptr(), buf.data_ptr(), n // 2, 0, 0, -1)), 2)
        table[n] = row
        log.info(f" all-reduce autotune {n} B: {row}")
    xg.ll_max_bytes, xg.twoshot_min_bytes = keep
    ok = xg.error() == 0
    ll_max, two_min, xgmi_max = comm_thresholds(table, cap)
    best = {n: min(v for k, v in r.items() if k != "rccl") for n, r in table.items()}
    xg.ll_max_bytes = ll_max
    xg.twoshot_min_bytes = two_min if two_min else cap + 16   # never, unless above the one-shot capacity
    tp.xgmi_max_ar = xgmi_max
    tp.comm_info.update({"allreduce_us": {str(k): v for k, v in table.items()}, "ll_max_bytes": ll_max,
                         "twoshot_min_bytes": two_min, "xgmi_max_bytes": xgmi_max,
                         "xgmi_allreduce_us": best.get(16384), "rccl_allreduce_us": table.get(16384, {}).get("rccl")})
    if not _agree(tp, ok) or xgmi_max == 0:
        tp.xgmi = None
    log.info(f" TP all-reduce transports (us): {table} -> LL <= {ll_max} B, two-shot >= {two_min} B, "
             f"xGMI <= {xgmi_max} B, RCCL above")
