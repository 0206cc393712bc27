"""Data parallelism over decision-engine replicas (BASELINE config 5: "half-node decision engine").

With ``WORLD_SIZE = replicas x tp`` (``engine.tp`` / ``K8S_TP``), ranks ``[r*tp, (r+1)*tp)`` form
replica ``r``: a complete tensor-parallel engine with its own weights, KV cache, RCCL communicator and
xGMI peer regions (``comm.init_from_env``).  Global rank 0 runs the control plane (the reference's
whole ``scheduler.py``) and the leader of replica 0.  The leader of every other replica serves chat
requests from rank 0 over a :class:`ReplicaLink`; its TP followers track its schedule through the
replica's ``ControlChannel``.

:class:`ReplicaRouterBackend` is the decision backend on rank 0.  Every request of a call goes to the
replica with the fewest requests in flight (ties rotate), so single-pod calls -- every call of the
``sequential`` and ``continuous`` scheduler modes -- spread over the replicas instead of staying on
replica 0.  Links are multiplexed: requests carry ids, a receiver thread on each side completes them as
they finish, and a remote leader hands every request to its engine's background serving loop, so the
remote replica batches continuously and any number of requests can be outstanding per link.  A failure
of any share raises, so retries / circuit breaker / fallback of the decision service see one failed
engine call, as for a single engine.  The reference has no counterpart (one remote HTTPS call per pod,
``scheduler.py:425-433``; pods detected one at a time, ``:662-681``).
"""

from __future__ import annotations

import datetime
import itertools
import logging
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from concurrent.futures import TimeoutError as FutureTimeout
from typing import Dict, List, Optional, Sequence

import torch.distributed as dist

from .comm import TPGroup

log = logging.getLogger(__name__)

_STOP = "__stop__"
_PING, _PONG = "__ping__", "__pong__"
# Gloo link timeout: a stalled but live peer fails the link within this many seconds instead of parking the receive
# threads for days (K8S_REPLICA_LINK_TIMEOUT_S; the engine watchdog's scale).  Idle links stay up through keepalives
# sent every quarter of it (rank 0 pings, the remote leader answers).
LINK_TIMEOUT_S = float(__import__("os").environ.get("K8S_REPLICA_LINK_TIMEOUT_S", "300"))


class ReplicaLink:
    """Rank 0 <-> the leader of one remote replica: two two-rank gloo groups, one per direction, each used by
    exactly one thread per side (so the collectives stay in the same order on both ranks).  Requests and replies
    carry ids: any number can be outstanding, replies arrive in completion order."""

    def __init__(self, replica: int, leader: int, down, up, timeout_s: float = LINK_TIMEOUT_S):
        self.replica = replica
        self.timeout_s = timeout_s
        self.leader = leader        # global rank of the remote replica's TP rank 0
        self.down = down            # rank 0 -> leader (requests, stop)
        self.up = up                # leader -> rank 0 (replies, stop acknowledgement)
        self._send_lock = threading.Lock()
        self._ids = itertools.count()
        self._pending: Dict[int, Future] = {}
        self._plock = threading.Lock()
        self._rx: Optional[threading.Thread] = None
        self.inflight = 0           # requests sent and not answered yet (router load)
        self.dead: Optional[str] = None   # set when the link failed: every later submit fails at once
        self._last_send = time.monotonic()
        self._ka: Optional[threading.Thread] = None
        self._closing = threading.Event()

    @staticmethod
    def _bcast(obj, src: int, group):
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=group)
        return box[0]

    # ---- rank-0 side
    def start(self) -> None:
        """Rank 0, once its engine is built (ReplicaRouterBackend does this): start the receive thread and the
        keepalive, whose first ping goes out at once -- the remote leader is parked in ``receive`` since ITS engine
        build, and an idle link must not let that wait reach the gloo timeout."""
        self._start_rx()

    def _start_rx(self) -> None:
        if self._rx is not None:
            return

        def run():
            why = f"replica {self.replica} link closed"
            try:
                while True:
                    msg = self._bcast(None, self.leader, self.up)
                    if msg == _STOP:
                        break
                    if msg == _PONG:
                        continue
                    with self._plock:
                        fut = self._pending.pop(msg["id"], None)
                    if fut is None:
                        continue
                    if "error" in msg:
                        fut.set_exception(RuntimeError(f"replica {self.replica}: {msg['error']}"))
                    else:
                        fut.set_result(list(msg["texts"]))
            except Exception as e:  # noqa: BLE001 -- the remote leader died or the gloo link broke
                why = f"replica {self.replica} link failed: {type(e).__name__}: {e}"
                log.error(f" {why}")
            self._close(why)

        self._rx = threading.Thread(target=run, name=f"replica{self.replica}-rx", daemon=True)
        self._rx.start()

        def keepalive():
            every = max(0.05, self.timeout_s / 4)
            first = True
            while first or not self._closing.wait(every / 4):
                if self.dead:
                    return
                if not first and time.monotonic() - self._last_send < every:
                    continue
                first = False
                try:
                    self._send(_PING)
                except Exception as e:  # noqa: BLE001
                    self._close(f"replica {self.replica} link failed on keepalive: {type(e).__name__}: {e}")
                    return

        self._ka = threading.Thread(target=keepalive, name=f"replica{self.replica}-keepalive", daemon=True)
        self._ka.start()

    def _send(self, obj) -> None:
        with self._send_lock:
            if self._closing.is_set() and obj is not _STOP:
                return
            self._bcast(obj, 0, self.down)
            self._last_send = time.monotonic()

    def _close(self, why: str) -> None:
        """Nothing more will be answered on this link: fail every pending future and every later submit."""
        with self._plock:
            self.dead = self.dead or why
            left, self._pending = self._pending, {}
        for fut in left.values():
            if not fut.done():
                fut.set_exception(RuntimeError(why))

    def submit(self, requests) -> Future:
        """Send a share of chat requests; the future resolves to their texts (request order), or fails when the
        link is (or becomes) dead."""
        self._start_rx()
        fut: Future = Future()
        rid = next(self._ids)
        fut.rid = rid   # type: ignore[attr-defined]  (cancel() takes it)
        n = len(requests)
        with self._plock:
            if self.dead:
                fut.set_exception(RuntimeError(self.dead))
                return fut
            self._pending[rid] = fut
            self.inflight += n

        def done(_f, n=n):
            with self._plock:
                self.inflight -= n

        fut.add_done_callback(done)
        try:
            self._send({"id": rid, "requests": list(requests)})
        except Exception as e:  # noqa: BLE001
            self._close(f"replica {self.replica} link failed on send: {type(e).__name__}: {e}")
        return fut

    def cancel(self, fut: Future, why: str) -> None:
        """Give up on a share (its caller's deadline passed): it leaves the pending table and the router's load
        figure at once; a late reply is dropped."""
        with self._plock:
            self._pending.pop(getattr(fut, "rid", None), None)
        if not fut.done():
            fut.set_exception(TimeoutError(why))

    def stop(self) -> None:
        self._start_rx()
        self._closing.set()
        self._send(_STOP)
        self._rx.join(timeout=120)

    # ---- leader side
    def receive(self):
        return self._bcast(None, 0, self.down)

    def reply(self, payload) -> None:
        with self._send_lock:
            self._bcast(payload, self.leader, self.up)


def make_replica_links(tp: TPGroup, timeout_s: float = LINK_TIMEOUT_S) -> List[ReplicaLink]:
    """Collective over the world (every rank must call it).  Rank 0 gets one link per remote
    replica, a remote leader gets its own link, every other rank an empty list.  Every link operation is bounded
    by ``timeout_s`` (idle links are kept alive by keepalives)."""
    links: List[ReplicaLink] = []
    if tp.replicas <= 1 or tp.simulate:
        return links
    me = tp.global_rank
    tmo = datetime.timedelta(seconds=timeout_s)
    for r in range(1, tp.replicas):
        leader = r * tp.world
        down = dist.new_group(ranks=[0, leader], backend="gloo", timeout=tmo)
        up = dist.new_group(ranks=[0, leader], backend="gloo", timeout=tmo)
        if me in (0, leader):
            links.append(ReplicaLink(r, leader, down, up, timeout_s))
    return links


class ReplicaRouterBackend:
    """Decision backend of rank 0 that sends every request to the least-loaded engine replica."""

    reply_grace_s = 5.0

    def __init__(self, local, links: Sequence[ReplicaLink]):
        self.local = local
        self.links = list(links)
        self.name = f"{getattr(local, 'name', 'local')}x{len(self.links) + 1}"
        self.dispatched = [0] * (len(self.links) + 1)
        self._local_inflight = 0
        self._lock = threading.Lock()
        self._cursor = 0
        for link in self.links:    # keepalives from now on, whether or not a request ever comes
            link.start()

    @property
    def replicas(self) -> int:
        return len(self.links) + 1

    @property
    def engine(self):
        """The local engine (start_backend_loop puts it in background mode for concurrent callers)."""
        return getattr(self.local, "engine", None)

    def _loads(self) -> List[int]:
        return [self._local_inflight] + [link.inflight for link in self.links]

    def assign(self, n: int) -> List[int]:
        """Replica of each of ``n`` requests: least in flight first, ties rotate (so serial single-request calls
        alternate over the replicas)."""
        with self._lock:
            loads = self._loads()
            out = []
            for _ in range(n):
                k = self.replicas
                best = min(range(k), key=lambda i: (loads[i], (i - self._cursor) % k))
                out.append(best)
                loads[best] += 1
                self._cursor = (best + 1) % k
            for i in out:
                self.dispatched[i] += 1
            self._local_inflight += out.count(0)
            return out

    def complete(self, requests) -> List[str]:
        where = self.assign(len(requests))
        shares: List[List[int]] = [[] for _ in range(self.replicas)]
        for j, i in enumerate(where):
            shares[i].append(j)
        # a remote share is waited for no longer than the call's deadline (plus a grace period for the reply),
        # counted from the start of the call, not from the end of the local share
        limits = [float(r.deadline_s) for r in requests if getattr(r, "deadline_s", None)]
        end = time.monotonic() + min(limits) + self.reply_grace_s if limits else None
        futs = {i: self.links[i - 1].submit([requests[j] for j in shares[i]])
                for i in range(1, self.replicas) if shares[i]}
        out: List[str] = [""] * len(requests)
        err: Optional[BaseException] = None
        try:
            if shares[0]:
                for j, text in zip(shares[0], self.local.complete([requests[j] for j in shares[0]])):
                    out[j] = text
        except BaseException as e:  # noqa: BLE001 -- the remote shares are still collected, then re-raised
            err = e
        finally:
            with self._lock:
                self._local_inflight -= len(shares[0])
        for i, fut in futs.items():
            try:
                left = None if end is None else max(0.0, end - time.monotonic())
                for j, text in zip(shares[i], fut.result(timeout=left)):
                    out[j] = text
            except FutureTimeout:
                why = f"replica {i} did not answer within the call deadline"
                self.links[i - 1].cancel(fut, why)
                err = err or TimeoutError(why)
            except BaseException as e:  # noqa: BLE001
                err = err or e
        if err is not None:
            raise err
        return out

    def shutdown(self) -> None:
        for link in self.links:
            try:
                link.stop()
            except Exception as e:  # noqa: BLE001
                log.warning(f" replica {link.replica} did not acknowledge shutdown: {e}")


def serve_replica(backend, link: ReplicaLink, engine=None, workers: int = 64) -> None:
    """Leader of a remote replica: hand every request share from rank 0 to the engine's background serving loop
    (so shares from concurrent rank-0 callers batch together), reply as each completes, until rank 0 sends stop;
    then release the replica's TP followers (``engine.shutdown_workers``)."""
    if engine is not None and hasattr(engine, "start_background"):
        engine.start_background()
    pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix=f"replica{link.replica}")

    def handle(msg):
        try:
            link.reply({"id": msg["id"], "texts": backend.complete(msg["requests"])})
        except Exception as e:  # noqa: BLE001 -- reported to rank 0, which decides (retry/fallback)
            link.reply({"id": msg["id"], "error": f"{type(e).__name__}: {e}"})

    try:
        while True:
            msg = link.receive()
            if msg == _STOP:
                break
            if msg == _PING:
                link.reply(_PONG)
                continue
            pool.submit(handle, msg)
        pool.shutdown(wait=True)
        link.reply(_STOP)
    finally:
        if engine is not None:
            if hasattr(engine, "stop_background"):
                engine.stop_background()
            engine.shutdown_workers()
