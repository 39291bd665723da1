"""Communication for the date-sharded step: the four exchanges ``pipeline.run_step`` makes
between date shards, behind one small interface so the same step code runs over

* ``TorchComm`` -- ``torch.distributed`` (RCCL over xGMI with backend "nccl" on the GPU
  box; gloo on CPU): one process per GPU, the production path;
* ``LocalComm`` -- N shards as N threads of ONE process on one device (tests): every
  exchange is a device-to-device copy ordered by HIP events, so the whole sharded step
  (halo send/recv, IC all-gather, exact Gram all-reduce) runs on the HIP kernels of a
  single MI355X and can be compared bit-for-bit with the 1-shard run.

Exchanges: point-to-point halo slabs to rank+1 (``exchange``: one
``batch_isend_irecv`` group of the rank's send and receive),
the daily IC series (``all_gather``) and the exact Gram limbs / pair counts
(``all_reduce_sum`` of int64 -- integer sums, so the reduction order is free).
"""
from __future__ import annotations

import threading

import torch
import torch.distributed as dist


class _HostRecv:
    """A receive staged through host memory: wait() copies it into the device tensor."""

    def __init__(self, req, host, out):
        self.req, self.host, self.out = req, host, out

    def wait(self):
        self.req.wait()
        self.out.copy_(self.host)


class TorchComm:
    """torch.distributed on the default process group (RCCL / gloo).  RCCL orders its
    transfers after the producing kernels of the current stream (and the current stream
    after the received data on wait()).  gloo does not order its point-to-point transfers of
    device tensors with the stream that produced them (a halo slab could be sent before
    torch.cat had written it: seen as a wrong halo at world 3 on one GPU), so with gloo every
    device tensor is staged through host memory: sends copy it out (stream-synchronous),
    receives land in host buffers copied in on wait(), collectives run on host copies.

    Consequence for timing: under gloo the staging copy blocks until the stream
    drains, so the halo exchange is synchronous and never overlaps the owned-date fused pass
    the step posts behind it -- gloo runs check correctness, not overlap.  Only the nccl
    (RCCL) backend, i.e. the driver's multi-GPU bench, exercises the overlapped ordering."""

    def __init__(self):
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.host_staged = dist.get_backend() == "gloo"

    def _stage(self, t):
        return t.cpu() if self.host_staged and t.is_cuda else t

    def isend(self, t, dst):
        return dist.isend(self._stage(t), dst)

    def irecv(self, t, src):
        if self.host_staged and t.is_cuda:
            host = torch.empty(t.shape, dtype=t.dtype)
            return _HostRecv(dist.irecv(host, src), host, t)
        return dist.irecv(t, src)

    def exchange(self, sends, recvs):
        """Point-to-point sends [(t, dst)] and receives [(t, src)] posted as ONE
        ``batch_isend_irecv`` group (RCCL coalesces the group's transfers); the returned
        requests are waited on by the caller."""
        ops, outs = [], []
        for t, d in sends:
            ops.append(dist.P2POp(dist.isend, self._stage(t), d))
        for t, s in recvs:
            if self.host_staged and t.is_cuda:
                host = torch.empty(t.shape, dtype=t.dtype)
                ops.append(dist.P2POp(dist.irecv, host, s))
                outs.append((host, t))
            else:
                ops.append(dist.P2POp(dist.irecv, t, s))
                outs.append(None)
        if not ops:
            return []
        reqs = dist.batch_isend_irecv(ops)
        nsend = len(sends)
        res = list(reqs[:nsend])
        for r, o in zip(reqs[nsend:], outs):
            res.append(_HostRecv(r, *o) if o is not None else r)
        return res

    def all_gather(self, t):
        src = self._stage(t.contiguous())
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src)
        return [p.to(t.device) for p in parts] if src is not t and t.is_cuda else parts

    def all_reduce_sum(self, t):
        if self.host_staged and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            t.copy_(h)
            return t
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def barrier(self):
        dist.barrier()


class _Done:
    def wait(self):
        return None


class _Recv:
    def __init__(self, hub, key, out):
        self.hub, self.key, self.out = hub, key, out

    def wait(self):
        t, ev = self.hub.take(self.key)
        if ev is not None:
            st = torch.cuda.current_stream(self.out.device)
            st.wait_event(ev)
            t.record_stream(st)                  # allocated on the sender's stream
        self.out.copy_(t)


class LocalHub:
    """Rendezvous of ``world`` in-process shards (one thread each)."""

    def __init__(self, world, timeout=300.0):
        self.world = world
        self.timeout = timeout
        self._cv = threading.Condition()
        self._mail = {}
        self._barrier = threading.Barrier(world, timeout=timeout)
        self._slots = [None] * world
        self.failed = False

    def abort(self):
        """A shard failed: wake every waiter (they raise instead of timing out)."""
        with self._cv:
            self.failed = True
            self._cv.notify_all()
        self._barrier.abort()

    def post(self, key, t):
        ev = None
        if t.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(t.device))
        with self._cv:
            self._mail.setdefault(key, []).append((t, ev))
            self._cv.notify_all()

    def take(self, key):
        with self._cv:
            ok = self._cv.wait_for(lambda: self.failed or self._mail.get(key), timeout=self.timeout)
            if self.failed:
                raise RuntimeError("LocalComm: another shard failed")
            if not ok:
                raise TimeoutError(f"LocalComm: no message for {key}")
            return self._mail[key].pop(0)

    def gather(self, rank, t):
        """Every rank's ``t`` (a private copy made on the caller's stream), rank order."""
        c = t.clone()
        ev = None
        if c.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(c.device))
        self._barrier.wait()                      # previous gather fully consumed
        self._slots[rank] = (c, ev)
        self._barrier.wait()                      # all deposited
        got = list(self._slots)
        self._barrier.wait()                      # all read the slot list
        out = []
        for x, e in got:
            if e is not None:
                st = torch.cuda.current_stream(x.device)
                st.wait_event(e)
                x.record_stream(st)              # allocated on the depositor's stream
            out.append(x.clone())                  # own copy, ordered after the producer
        return out


class LocalComm:
    """One shard's endpoint on a LocalHub (same interface as TorchComm)."""

    def __init__(self, hub: LocalHub, rank: int):
        self.hub, self.rank, self.world = hub, rank, hub.world
        self._n = {}

    def _key(self, src, dst):
        k = (src, dst)
        self._n[k] = self._n.get(k, 0) + 1
        return (src, dst, self._n[k])

    def isend(self, t, dst):
        self.hub.post(self._key(self.rank, dst), t.clone())
        return _Done()

    def irecv(self, t, src):
        return _Recv(self.hub, self._key(src, self.rank), t)

    def exchange(self, sends, recvs):
        return [self.isend(t, d) for t, d in sends] + [self.irecv(t, s) for t, s in recvs]

    def all_gather(self, t):
        return self.hub.gather(self.rank, t.contiguous())

    def all_reduce_sum(self, t):
        parts = self.hub.gather(self.rank, t.contiguous())
        acc = parts[0]
        for p in parts[1:]:
            acc += p
        t.copy_(acc)
        return t

    def barrier(self):
        self.hub._barrier.wait()


def run_local_shards(world, fn, timeout=600.0):
    """Run ``fn(rank, comm)`` for ``world`` in-process shards on threads; each thread runs
    on its own HIP stream when a GPU is present.  Returns the per-rank results and re-raises
    the first shard's exception."""
    hub = LocalHub(world, timeout=timeout)
    res = [None] * world
    err = [None] * world

    def body(r):
        try:
            if torch.cuda.is_available():
                with torch.cuda.stream(torch.cuda.Stream()):
                    res[r] = fn(r, LocalComm(hub, r))
                    torch.cuda.current_stream().synchronize()
            else:
                res[r] = fn(r, LocalComm(hub, r))
        except BaseException as e:  # noqa: BLE001 -- reported to the caller below
            err[r] = e
            hub.abort()

    th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    for e in err:      # the original failure, not the other shards' aborted waits
        if e is not None and not isinstance(e, threading.BrokenBarrierError) and "another shard" not in str(e):
            raise e
    for e in err:
        if e is not None:
            raise e
    if any(t.is_alive() for t in th):
        raise TimeoutError("LocalComm shards did not finish")
    return res
