"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL ("nccl" on ROCm).

Two exchange steps exist on the hot path:
  * training: gradients are summed over ranks once per optimizer step (on the iter_size
    accumulation boundary of module.py:235-243), by ``GradientBuckets`` (a few large
    asynchronous bucket all-reduces launched from backward's gradient hooks, used by
    train.PatchClassificationStep and bench.py's multi-GPU step);
  * push: images are independent, so each rank scans a contiguous shard and one MIN
    all-reduce over packed 64-bit keys (distance bits << 32 | image index) reproduces the
    serial scan's "strictly smaller, earlier image wins" order exactly (push.py:101, 265);
    the owner of each winning key then contributes the feature vector / patch index.
The reference itself has no collectives (every config sets Trainer.gpus = 1).
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

INT32_MAX = 2 ** 31 - 1


def world_info(group=None) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) shard of n items; shard sizes differ by at most one."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, int]:
    """Initialises the default process group from torchrun's env (RANK/WORLD_SIZE/...).
    Returns (rank, local_rank, world_size); a no-op single process without those vars."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)
    return rank, local_rank, world


def reduce_push_state(state, group=None) -> None:
    """Merges per-rank push minima into the global one, identically on every rank."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    bits = state.dist.contiguous().view(torch.int32).to(torch.int64)  # d >= 0 (relu) or +inf
    img = torch.where(state.img >= 0, state.img, torch.full_like(state.img, INT32_MAX))
    key = (bits << 32) | img
    gkey = key.clone()
    dist.all_reduce(gkey, op=dist.ReduceOp.MIN, group=group)
    mine = (key == gkey) & (state.img >= 0)
    fmap = torch.where(mine[:, None], state.fmap, torch.zeros_like(state.fmap))
    patch = torch.where(mine, state.patch.to(torch.int64) + 1, torch.zeros_like(img))
    dist.all_reduce(fmap, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(patch, op=dist.ReduceOp.SUM, group=group)
    if state.second is not None:
        # global runner-up: the winning rank offers its own runner-up, every other rank its best
        cand = torch.where(mine, state.second, torch.minimum(state.dist, state.second))
        dist.all_reduce(cand, op=dist.ReduceOp.MIN, group=group)
        state.second.copy_(cand)
    # geometry (H, W, h, w) of each prototype's winning image, for its rf box (push.py:288-307):
    # the owner rank's row of a [P, 4] tensor, summed over ranks (a plain collective, no pickles)
    mine_rows = torch.nonzero(mine).flatten().tolist()
    own_img = state.img.cpu()
    geo = torch.zeros((mine.shape[0], 4), dtype=torch.int64)
    for j in mine_rows:
        geo[j] = torch.tensor(state.geometry[int(own_img[j])], dtype=torch.int64)
    geo = geo.to(mine.device)
    dist.all_reduce(geo, op=dist.ReduceOp.SUM, group=group)
    gimg = gkey & 0xFFFFFFFF
    state.dist.copy_((gkey >> 32).to(torch.int32).view(torch.float32))
    state.img.copy_(torch.where(gimg == INT32_MAX, torch.full_like(gimg, -1), gimg))
    state.patch.copy_((patch - 1).to(torch.int32))
    state.fmap.copy_(fmap)
    won = state.img.cpu().tolist()
    geo_h = geo.cpu().tolist()
    for j, im in enumerate(won):
        if im >= 0:
            state.geometry[int(im)] = tuple(int(v) for v in geo_h[j])


def reduce_bound_boxes(boxes, device="cpu", group=None):
    """Merges per-rank push bound boxes (push.py:338-343): each rank fills the rows of the
    prototypes whose winning image lies in its shard and leaves -1 elsewhere, so one MAX
    all-reduce gives every rank the full table. Returns a numpy int64 array."""
    import numpy as np
    t = torch.as_tensor(np.asarray(boxes, dtype=np.int64), device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.cpu().numpy()


class GradientBuckets:
    """Sums (or averages) the .grad of ``params`` over ranks with a few large asynchronous
    all-reduces — the exchange step of data-parallel training (train.PatchClassificationStep,
    and bench.py's multi-GPU step).

    Buckets are filled in reverse registration order (the order backward produces grads), each
    up to ``bucket_mb`` MiB of one dtype; xGMI rings are per-link bound, so few large collectives
    beat many small ones. ``arm()`` before the backward of the step that ends a gradient
    accumulation (module.py:235-243: the optimizer steps every iter_size micro-steps) makes each
    bucket's all-reduce start from the gradient hook of its last parameter, so the exchange
    overlaps the rest of the backward; buckets are always launched in index order, so every rank
    issues the same collective sequence. Without ``arm()``, ``allreduce()`` + ``wait()`` do the
    same after backward.

    Each bucket owns one persistent flat buffer, and after its first exchange every gradient of
    the bucket IS a view into it (DDP's gradient-as-bucket-view): backward accumulates straight
    into the buffer, the all-reduce runs on it in place and the reduced values are already where
    ``p.grad`` points, so an exchange is one collective (+ the averaging scale) per bucket, with
    no concatenation copy and no device -> host read. Zeroing the gradients in place
    (``zero_grad(set_to_none=False)``, the reference's torch-1.10 default) keeps the views.

    A parameter that got no gradient on a rank contributes zeros there, and it gets the reduced
    gradient on every rank when any rank had one (a had-gradient flag per parameter is summed
    with the bucket), so no replica skips an update the others make. Only then is a flag read
    on the host: for parameters whose local gradient is None.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_mb: float = 64.0, group=None,
                 average: bool = True):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.average = average
        limit = int(bucket_mb * 2 ** 20)
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            nbytes = p.numel() * p.element_size()
            if cur and (size + nbytes > limit or p.dtype != cur[0].dtype or p.device != cur[0].device):
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {id(p): b for b, bucket in enumerate(self.buckets) for p in bucket}
        self._numel = [sum(p.numel() for p in bucket) for bucket in self.buckets]
        self._flat: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        self._hooks = []
        self._armed = False
        self._ready = [0] * len(self.buckets)
        self._pending: List[Optional[tuple]] = [None] * len(self.buckets)
        self._next = 0

    def _world(self) -> int:
        return world_info(self.group)[1]

    def arm(self) -> None:
        """Launch each bucket's all-reduce from backward's gradient hooks (next backward only)."""
        if self._world() == 1:
            return
        if not self._hooks:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._ready = [0] * len(self.buckets)
        self._armed = True

    def _on_grad(self, p) -> None:
        if not self._armed:
            return
        b = self._bucket_of[id(p)]
        self._ready[b] += 1
        while self._next < len(self.buckets) and self._ready[self._next] == len(self.buckets[self._next]):
            self._launch(self._next)

    def flat(self, b: int) -> torch.Tensor:
        """Bucket b's persistent buffer: the parameters' gradients in bucket order, then one
        had-gradient flag per parameter."""
        if self._flat[b] is None:
            ref = self.buckets[b][0]
            self._flat[b] = torch.zeros(self._numel[b] + len(self.buckets[b]), dtype=ref.dtype, device=ref.device)
        return self._flat[b]

    def bind_grads(self) -> None:
        """Make every parameter's .grad a view into its bucket's buffer now (existing values
        copied; None becomes zeros): a caller whose kernels write gradients into fixed buffers
        (bench.py's captured step) then writes them straight into the exchange buffers."""
        for b, bucket in enumerate(self.buckets):
            flat, off = self.flat(b), 0
            for p in bucket:
                n = p.numel()
                seg = flat[off:off + n]
                if p.grad is None:
                    seg.zero_()
                elif p.grad.data_ptr() != seg.data_ptr():
                    seg.copy_(p.grad.reshape(-1))
                p.grad = seg.view_as(p)
                off += n

    def _launch(self, b: int) -> None:
        bucket, flat = self.buckets[b], self.flat(b)
        n_total = self._numel[b]
        missing, off = [], 0
        for i, p in enumerate(bucket):
            n = p.numel()
            seg = flat[off:off + n]
            g = p.grad
            if g is None:
                seg.zero_()
                missing.append(i)
            elif g.data_ptr() != seg.data_ptr() or g.shape != p.shape:
                seg.copy_(g.reshape(-1))   # first exchange (or a replaced .grad): alias it from now on
                p.grad = seg.view_as(p)
            off += n
        flags = flat[n_total:]
        flags.fill_(1.0)
        for i in missing:
            flags[i:i + 1].zero_()
        work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._pending[b] = (work, missing)
        self._next = b + 1

    def allreduce(self) -> None:
        """Launch every bucket not yet launched (in index order)."""
        if self._world() == 1:
            return
        while self._next < len(self.buckets):
            self._launch(self._next)

    def wait(self) -> None:
        """Completes the exchange on the current stream (no host synchronisation unless a
        parameter's local gradient is None)."""
        world = self._world()
        if world == 1:
            return
        self.allreduce()
        for b, bucket in enumerate(self.buckets):
            work, missing = self._pending[b]
            work.wait()
            flat = self._flat[b]
            if self.average:
                flat.div_(world)
            if missing:  # some rank may have had a gradient for a parameter this rank lacks
                had = flat[self._numel[b]:][missing].tolist()
                offs = [0]
                for p in bucket:
                    offs.append(offs[-1] + p.numel())
                for i, h in zip(missing, had):
                    if h > 0:  # every rank takes the reduced gradient; otherwise none has one
                        bucket[i].grad = flat[offs[i]:offs[i + 1]].view_as(bucket[i])
        self._pending = [None] * len(self.buckets)
        self._next = 0
        self._armed = False

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
