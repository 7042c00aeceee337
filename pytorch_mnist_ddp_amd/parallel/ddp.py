"""DistributedDataParallel (reference mnist_ddp.py:173: ``DistributedDataParallel(model, device_ids=[gpu])``).

Semantics reproduced from torch DDP (torch/nn/parallel/distributed.py, reducer.hpp):

* construction: verify every rank has the same parameter shapes (all-gather of a shape digest),
  then broadcast rank 0's parameters and buffers, coalesced (``_sync_module_states``);
* gradient buckets: parameters in *reverse* registration order (= backward ready order), a new
  bucket whenever the running size reaches the cap; first bucket capped at ``first_bucket_cap_mb``
  (1 MiB), then ``bucket_cap_mb`` (25 MiB).  For the reference Net this yields exactly torch's
  rebuilt layout: {fc2.b, fc2.w, fc1.b, fc1.w} (4,724,264 B) and {conv2.*, conv1.*} (75,264 B);
* backward: a post-accumulate-grad hook per parameter copies ``grad / world_size`` into its
  bucket; when a bucket is complete its all-reduce(SUM) is launched asynchronously, overlapping
  the rest of backward; a finalize callback queued on the autograd engine waits for the works and
  copies the averaged buckets back into ``.grad``;
* ``state_dict()`` keys carry the ``module.`` prefix; ``no_sync()`` skips reduction.

Transport: ``torch.distributed`` (``nccl`` = RCCL on ROCm, ``gloo`` on CPU), or - given the
framework's own RCCL communicator (``comm=``) and device parameters - the native C++ reducer
(:class:`NativeBucketReducer` over ``csrc/runtime/bucket_reducer.cpp``).  The fused training engine does not use these
hooks - it reduces the flat gradient buffer in two buckets from C++ (``csrc/runtime/engine.cpp``)
and the wrapper then only provides DDP's construction / state_dict semantics (``engine_managed``).
"""
from __future__ import annotations

import contextlib
import hashlib

import torch
import torch.distributed as dist
import torch.nn as nn


def compute_bucket_assignment(sizes_bytes: list[int], caps_bytes: list[int]) -> list[list[int]]:
    """Greedy bucket assignment over tensors given in *ready order* (indices into ``sizes_bytes``).

    Mirrors c10d ``compute_bucket_assignment_by_size``: a bucket is closed as soon as its size
    reaches the current cap; the caps list is walked (last cap repeats).
    """
    buckets, cur, cur_size, li = [], [], 0, 0
    for i, sz in enumerate(sizes_bytes):
        cur.append(i)
        cur_size += sz
        if cur_size >= caps_bytes[min(li, len(caps_bytes) - 1)]:
            buckets.append(cur)
            cur, cur_size = [], 0
            li += 1
    if cur:
        buckets.append(cur)
    return buckets


# Net parameter indices (registration order): conv1.w, conv1.b, conv2.w, conv2.b, fc1.w, fc1.b, fc2.w, fc2.b
_FC_PARAMS, _CONV_PARAMS = frozenset({4, 5, 6, 7}), frozenset({0, 1, 2, 3})


def engine_bucket_layout(bucket_indices: list[list[int]]) -> bool:
    """Map a DDP bucket assignment of the reference ``Net`` onto the fused engine's schedules:
    True = two buckets {fc2.*, fc1.*} then {conv2.*, conv1.*} (torch DDP's rebuilt layout at the
    default caps), False = one bucket over every gradient (e.g. a first-bucket cap
    >= 4.5 MiB).  Any other layout raises: the engine's buckets are fixed kernels, so a layout it
    cannot run is refused instead of silently ignored (``--engine module`` runs any layout)."""
    sets = [frozenset(b) for b in bucket_indices]
    if sets == [_FC_PARAMS, _CONV_PARAMS]:
        return True
    if sets == [_FC_PARAMS | _CONV_PARAMS]:
        return False
    raise ValueError(f"the fused engine runs the DDP bucket layouts {{fc}},{{conv}} (default caps) and a single "
                     f"bucket; --bucket-cap-mb/--first-bucket-mb give {[sorted(b) for b in bucket_indices]} "
                     f"(parameter indices) - use --engine module for arbitrary buckets")


class BucketReducer:
    def __init__(self, params: list[torch.Tensor], buckets: list[list[int]], world_size: int,
                 process_group=None, comm=None):
        self.params = params
        self.world = world_size
        self.pg = process_group
        self.comm = comm
        self.bucket_of = {}
        self.buffers, self.offsets = [], []
        for b, idxs in enumerate(buckets):
            n = sum(params[i].numel() for i in idxs)
            p0 = params[idxs[0]]
            self.buffers.append(torch.zeros(n, dtype=p0.dtype, device=p0.device))
            offs, o = {}, 0
            for i in idxs:
                offs[i] = o
                o += params[i].numel()
                self.bucket_of[i] = b
            self.offsets.append(offs)
        self.buckets = buckets
        self._pending = [len(b) for b in buckets]
        self._works = [None] * len(buckets)
        self._armed = False
        self.enabled = True
        self.calls = []          # (bucket, numel) log of launched all-reduces, for tests/telemetry

    def prepare_for_backward(self) -> None:
        self._pending = [len(b) for b in self.buckets]
        self._works = [None] * len(self.buckets)
        self._armed = False

    def _launch(self, b: int) -> None:
        buf = self.buffers[b]
        self.calls.append((b, buf.numel()))
        if self.comm is not None and buf.is_cuda:
            self.comm.allreduce_sum(buf.data_ptr(), buf.numel(), 0 if buf.dtype == torch.float32 else 1,
                                    torch.cuda.current_stream().cuda_stream)
            self._works[b] = None
        else:
            self._works[b] = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def mark_ready(self, i: int) -> None:
        if not self.enabled:
            return
        if not self._armed:
            self._armed = True
            torch.autograd.Variable._execution_engine.queue_callback(self.finalize)
        b = self.bucket_of[i]
        p = self.params[i]
        off = self.offsets[b][i]
        view = self.buffers[b][off:off + p.numel()]
        if p.grad is None:
            view.zero_()
        else:
            torch.mul(p.grad.reshape(-1), 1.0 / self.world, out=view)     # pre-divide like DDP
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def finalize(self) -> None:
        for b, idxs in enumerate(self.buckets):
            if self._pending[b] != 0:            # some params got no grad this iteration
                for i in idxs:
                    if self.params[i].grad is None:
                        off = self.offsets[b][i]
                        self.buffers[b][off:off + self.params[i].numel()].zero_()
                self._pending[b] = 0
                self._launch(b)
            w = self._works[b]
            if w is not None:
                w.wait()
            for i in idxs:
                p = self.params[i]
                off = self.offsets[b][i]
                g = self.buffers[b][off:off + p.numel()].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
        self._armed = False


class NativeBucketReducer:
    """Adapter over the C++ ``_C.BucketReducer`` (csrc/runtime/bucket_reducer.cpp): same interface as
    :class:`BucketReducer`, but the copy-in, the RCCL all-reduce on a high-priority comm stream
    and the copy-out are enqueued from C++ with HIP events - no Python on the reduction path
    beyond the hook dispatch itself."""

    def __init__(self, params: list[torch.Tensor], buckets: list[list[int]], world_size: int, comm):
        from ..ops import native
        C = native.load()
        self.params = params
        self.world = world_size
        self.buckets = buckets
        self.slot = {}
        for b, idxs in enumerate(buckets):
            for s, i in enumerate(idxs):
                self.slot[i] = (b, s)
        self.impl = C.BucketReducer([[params[i].numel() for i in idxs] for idxs in buckets], world_size, comm)
        self._armed = False
        self._seen = set()
        self.enabled = True
        self.calls = []

    def prepare_for_backward(self) -> None:
        self.impl.prepare()
        self._armed = False
        self._seen = set()

    def mark_ready(self, i: int) -> None:
        if not self.enabled:
            return
        self._seen.add(i)
        if not self._armed:
            self._armed = True
            torch.autograd.Variable._execution_engine.queue_callback(self.finalize)
        b, s = self.slot[i]
        p = self.params[i]
        g = p.grad
        ptr = g.data_ptr() if g is not None else 0
        if g is not None and (not g.is_contiguous() or g.dtype != torch.float32):
            raise RuntimeError("native DDP reducer expects contiguous fp32 gradients")
        self.impl.mark_ready(b, s, ptr, ptr, torch.cuda.current_stream(p.device).cuda_stream)
        self._log_launches()

    def _log_launches(self) -> None:
        # buckets leave in index order every iteration, so launch k is bucket k % num_buckets
        for k in range(len(self.calls), self.impl.launches):
            nb = k % len(self.buckets)
            self.calls.append((nb, self.impl.bucket_numel(nb)))

    def finalize(self) -> None:
        dev = self.params[0].device
        stream = torch.cuda.current_stream(dev).cuda_stream
        for i, p in enumerate(self.params):      # parameters without a gradient contribute zeros
            if i not in self._seen:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                b, s = self.slot[i]
                self.impl.mark_ready(b, s, 0, p.grad.data_ptr(), stream)
        self._log_launches()
        self.impl.finalize(stream)
        self._log_launches()
        self._armed = False


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None, broadcast_buffers: bool = True,
                 process_group=None, bucket_cap_mb: float | None = None, find_unused_parameters: bool = False,
                 first_bucket_cap_mb: float = 1.0, comm=None, engine_managed: bool = False):
        super().__init__()
        if not dist.is_available() or not dist.is_initialized():
            raise RuntimeError("DistributedDataParallel requires an initialised default process group")
        self.module = module
        self.device_ids = device_ids
        self.process_group = process_group
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.world_size = dist.get_world_size(process_group)
        self.engine_managed = engine_managed
        params = [p for p in module.parameters() if p.requires_grad]
        self._verify_shapes(params)
        if not engine_managed:
            self._sync_module_states()
        # engine_managed: the fused engine broadcasts rank 0's parameters itself, over its own
        # transport, once that exists (FusedTrainer.broadcast_params) - a broadcast here would make
        # ProcessGroupNCCL build a communicator only for it
        cap = (25.0 if bucket_cap_mb is None else bucket_cap_mb) * 1024 * 1024
        first = first_bucket_cap_mb * 1024 * 1024
        ready_order = list(reversed(range(len(params))))
        sizes = [params[i].numel() * params[i].element_size() for i in ready_order]
        assignment = compute_bucket_assignment(sizes, [int(first), int(cap)])
        self.bucket_indices = [[ready_order[j] for j in b] for b in assignment]
        self.reducer = None
        if not engine_managed:
            if comm is not None and params and params[0].is_cuda:
                self.reducer = NativeBucketReducer(params, self.bucket_indices, self.world_size, comm)
            else:
                self.reducer = BucketReducer(params, self.bucket_indices, self.world_size, process_group, comm)
            for i, p in enumerate(params):
                p.register_post_accumulate_grad_hook(lambda _p, i=i: self.reducer.mark_ready(i))

    # ------------------------------------------------------------------ construction-time sync
    def _verify_shapes(self, params) -> None:
        digest = hashlib.sha1(repr([tuple(p.shape) for p in params]).encode()).digest()[:8]
        if self.engine_managed:                  # host collective over the store (no device comm)
            from .hostcomm import get_hostcomm
            if not get_hostcomm().all_equal(digest):
                raise RuntimeError("DDP: parameter shapes differ across ranks")
            return
        mine = torch.tensor([int.from_bytes(digest, "little", signed=True)], dtype=torch.int64)
        dev = params[0].device if params and dist.get_backend(self.process_group) == "nccl" else torch.device("cpu")
        mine = mine.to(dev)
        allv = [torch.zeros_like(mine) for _ in range(self.world_size)]
        dist.all_gather(allv, mine, group=self.process_group)
        if any(int(v.item()) != int(mine.item()) for v in allv):
            raise RuntimeError("DDP: parameter shapes differ across ranks")

    @torch.no_grad()
    def _sync_module_states(self) -> None:
        tensors = [p.data for p in self.module.parameters()] + [b.data for b in self.module.buffers()]
        if not tensors:
            return
        flat = torch.cat([t.reshape(-1) for t in tensors])
        src = dist.get_global_rank(self.process_group, 0) if self.process_group is not None else 0
        if flat.is_cuda and dist.get_backend(self.process_group) != "nccl":
            host = flat.cpu()                    # gloo bootstrap on GPU ranks: stage through the host
            dist.broadcast(host, src=src, group=self.process_group)
            flat.copy_(host)
        else:
            dist.broadcast(flat, src=src, group=self.process_group)
        o = 0
        for t in tensors:
            t.copy_(flat[o:o + t.numel()].view_as(t))
            o += t.numel()

    # ------------------------------------------------------------------ forward
    def forward(self, *inputs, **kwargs):
        if self.broadcast_buffers:
            bufs = list(self.module.buffers())
            if bufs:
                flat = torch.cat([b.reshape(-1) for b in bufs])
                dist.broadcast(flat, src=0, group=self.process_group)
        if self.reducer is not None and torch.is_grad_enabled():
            self.reducer.prepare_for_backward()
        return self.module(*inputs, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        prev = self.reducer.enabled if self.reducer else None
        if self.reducer:
            self.reducer.enabled = False
        try:
            yield
        finally:
            if self.reducer:
                self.reducer.enabled = prev


# ---------------------------------------------------------------------------- desync detection
def params_fingerprint(tensors) -> torch.Tensor:
    """Bit-exact fingerprint of fp32 tensors: int64 sums of their raw int32 bit patterns (plain and
    position-weighted), so any single-bit difference between ranks changes it."""
    parts = []
    for t in tensors:
        b = t.detach().reshape(-1).contiguous().view(torch.int32).to(torch.int64)
        w = torch.arange(b.numel(), device=b.device, dtype=torch.int64) % 8191 + 1
        parts.append(torch.stack([b.sum(), (b * w).sum()]))
    return torch.stack(parts).sum(0)


def params_fingerprint_host(tensors) -> bytes:
    """The same kind of fingerprint computed on the host from a D2H copy: startup paths use it so no
    torch GPU kernel (and its first-launch code-object load) runs inside the reference timer."""
    import numpy as np
    b_sum = w_sum = 0
    for t in tensors:
        h = t.detach().reshape(-1).contiguous().cpu().numpy().view(np.int32).astype(np.int64)
        w = np.arange(h.size, dtype=np.int64) % 8191 + 1
        b_sum += int(h.sum())
        w_sum += int((h * w).sum())
    return f"{b_sum}:{w_sum}".encode()


def assert_params_in_sync(tensors) -> None:
    """SURVEY §5.2 'DDP desync detector': every rank's parameters must be bitwise identical.

    The fingerprints are computed on the host and compared over the c10d store (``hostcomm``), so
    the check never creates a device communicator - on the nccl backend a ``dist.all_gather`` would
    build ProcessGroupNCCL's RCCL communicator next to the engine's own."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    from .hostcomm import get_hostcomm
    allv = get_hostcomm().gather_strings(params_fingerprint_host(tensors).decode())
    bad = [r for r, v in enumerate(allv) if v != allv[0]]
    if bad:
        raise RuntimeError(f"DDP desync: parameters on ranks {bad} differ from rank 0")

