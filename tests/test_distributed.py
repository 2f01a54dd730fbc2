"""CPU, world_size 2 over gloo: the sharded-push reduction equals the serial scan, and the
bucketed gradient all-reduce averages exactly."""
import math
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from protoseg_amd.distributed import GradientBuckets, reduce_bound_boxes, reduce_push_state, shard_bounds
from protoseg_amd.push import PushState


def _free_port():
    """A fresh rendezvous file for init_method='file://' (name kept from the TCP version)."""
    import tempfile
    fd, path = tempfile.mkstemp(prefix="protoseg_gloo_")
    os.close(fd)
    os.unlink(path)
    return path


def _serial_truth(per_image):
    """Strict '<' in image order over (dist, patch, fmap) per image and prototype; runner-up =
    the second smallest of every image's (best, runner-up) distances."""
    n_img, P = len(per_image), per_image[0][0].shape[0]
    best = [math.inf] * P
    img = [-1] * P
    patch = [-1] * P
    fmap = [None] * P
    for i in range(n_img):
        d, q, f, _ = per_image[i]
        for j in range(P):
            if float(d[j]) < best[j]:
                best[j], img[j], patch[j], fmap[j] = float(d[j]), i, int(q[j]), f[j]
    second = [sorted([float(im[0][j]) for im in per_image] + [float(im[3][j]) for im in per_image])[1]
              for j in range(P)]
    return best, img, patch, fmap, second


def _make_images(n_img, P, C):
    gen = torch.Generator().manual_seed(7)
    out = []
    for i in range(n_img):
        d = torch.randint(0, 6, (P,), generator=gen).float() / 4  # many exact ties across images
        d[torch.rand(P, generator=gen) < 0.2] = math.inf            # class absent in this image
        q = torch.randint(0, 500, (P,), generator=gen, dtype=torch.int32)
        f = torch.rand(P, C, generator=gen)
        d2 = d + torch.randint(0, 3, (P,), generator=gen).float() / 8  # the image's runner-up
        out.append((d, q, f, d2))
    return out


def _wire(obj):
    """Tensors -> numpy (pickled by value): a tensor put on a multiprocessing queue travels as a
    shared-memory handle that dies with the sending rank, which may exit before the parent reads."""
    if isinstance(obj, torch.Tensor):
        return ("__t", obj.detach().cpu().numpy().copy())
    if isinstance(obj, (list, tuple)):
        return type(obj)(_wire(o) for o in obj)
    return obj


def _unwire(obj):
    if isinstance(obj, tuple) and len(obj) == 2 and isinstance(obj[0], str) and obj[0] == "__t":
        return torch.from_numpy(obj[1])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_unwire(o) for o in obj)
    return obj


def _worker(rank, world, port, n_img, P, C, result_q):
    # file rendezvous (no TCP port to race for) and gloo's pair sockets on loopback
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        images = _make_images(n_img, P, C)
        lo, hi = shard_bounds(n_img, rank, world)
        st = PushState.create(P, C, "cpu")
        for i in range(lo, hi):  # host emulation of the device merge for this rank's shard
            d, q, f, d2 = images[i]
            better = d < st.dist
            st.second = torch.where(better, torch.minimum(st.dist, d2), torch.minimum(st.second, d))
            st.dist = torch.where(better, d, st.dist)
            st.img = torch.where(better, torch.full_like(st.img, i), st.img)
            st.patch = torch.where(better, q, st.patch)
            st.fmap = torch.where(better[:, None], f, st.fmap)
            st.geometry[i] = (8, 8, 2, 2)
        reduce_push_state(st)
        # gradient buckets: rank-dependent grads, tiny buckets to force several collectives
        params = [torch.nn.Parameter(torch.zeros(n)) for n in (5, 300, 17)]
        for k, p in enumerate(params):
            p.grad = torch.full_like(p, float(rank + 1) * (k + 1))
        gb = GradientBuckets(params, bucket_mb=1e-3)
        gb.allreduce()
        gb.wait()
        grads = [p.grad.clone() for p in params]
        # a parameter with a gradient on rank 1 only (data-dependent use), and one on neither:
        # the first gets the reduced gradient on EVERY rank, the second stays None everywhere
        extra = [torch.nn.Parameter(torch.zeros(4)), torch.nn.Parameter(torch.zeros(3))]
        extra[0].grad = torch.full((4,), 6.0) if rank == 1 else None
        gb2 = GradientBuckets(extra, bucket_mb=1.0)
        gb2.arm()  # hook path: rank 0 never fires extra[0]'s hook, so wait() launches the bucket
        gb2.wait()
        skipped = (None if extra[0].grad is None else extra[0].grad.clone(), extra[1].grad)
        # bound boxes: rank r owns the prototypes whose winning image lies in its shard
        boxes = torch.full((P, 6), -1, dtype=torch.int64)
        for j in range(P):
            if lo <= int(st.img[j]) < hi:
                boxes[j] = torch.tensor([int(st.img[j]), j, j + 3, 2 * j, 2 * j + 5, j % 4])
        merged = reduce_bound_boxes(boxes.numpy())
        # every prototype's winning image has its geometry on every rank (rf boxes)
        geo_ok = all(st.geometry.get(int(i)) == (8, 8, 2, 2) for i in st.img.tolist() if i >= 0)
        result_q.put(_wire((rank, st.dist, st.img, st.patch, st.fmap, geo_ok, grads, len(gb.buckets), merged,
                            st.second, skipped)))
        dist.barrier()  # neither rank tears gloo down while the other is still in a collective
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_img", [5, 8])
def test_sharded_push_reduction_equals_serial_scan(n_img):
    world, P, C = 2, 23, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_img, P, C, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [_unwire(q.get(timeout=120)) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    best, img, patch, fmap, second = _serial_truth(_make_images(n_img, P, C))
    for rank, d, im, pa, fm, ngeo, grads, nbuckets, boxes, sec, skipped in results:
        assert skipped[0] is not None and torch.equal(skipped[0], torch.full((4,), 3.0))  # (0 + 6) / 2
        assert skipped[1] is None
        assert sec.tolist() == second  # the sharded runner-up equals the serial one
        assert ngeo  # winners' geometry reached every rank
        for j in range(P):  # every rank holds the union of the per-shard bound boxes
            exp = [-1] * 6 if img[j] < 0 else [img[j], j, j + 3, 2 * j, 2 * j + 5, j % 4]
            assert list(boxes[j]) == exp
        for j in range(P):
            if img[j] < 0:
                assert im[j].item() == -1 and math.isinf(d[j].item())
                continue
            assert (d[j].item(), im[j].item(), pa[j].item()) == (best[j], img[j], patch[j])
            assert torch.equal(fm[j], fmap[j])
        assert nbuckets == 3
        for k, g in enumerate(grads):
            assert torch.allclose(g, torch.full_like(g, 1.5 * (k + 1)))  # mean of rank+1 over 2 ranks


def _bucket_view_worker(rank, world, port, result_q):
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.rand(5, 3)), torch.nn.Parameter(torch.rand(7)),
                  torch.nn.Parameter(torch.rand(4, 4))]
        gb = GradientBuckets(params, bucket_mb=100 / 2 ** 20, average=True)  # 2 buckets (64 + 28 B, 60 B)
        rounds = []
        for step in range(3):
            for p in params:  # zero_grad(set_to_none=False) after the first step: views survive
                if p.grad is not None:
                    p.grad.zero_()
            loss = sum(((rank + 1) * (step + 1) * p * torch.arange(p.numel()).view_as(p)).sum() for p in params)
            gb.arm()
            loss.backward()
            gb.wait()
            in_flat = all(any(f is not None and f.data_ptr() <= p.grad.data_ptr() < f.data_ptr() + f.numel() * 4
                              for f in gb._flat) for p in params)
            rounds.append(([p.grad.tolist() for p in params], in_flat))  # plain lists: no shared memory
        result_q.put((rank, rounds, len(gb.buckets)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gradient_buckets_alias_grads_across_steps():
    """After the first exchange every .grad is a view into its bucket's persistent buffer, and
    later steps (gradients zeroed in place, accumulated by backward into the buffer) reduce
    correctly with no copy: mean over ranks of (rank + 1) * (step + 1) * arange."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_view_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    mean = sum(r + 1 for r in range(world)) / world
    for rank, rounds, nb in results:
        assert nb == 2
        for step, (grads, in_flat) in enumerate(rounds):
            assert in_flat
            for g, shape in zip(grads, [(5, 3), (7,), (4, 4)]):
                g = torch.tensor(g)
                ref = mean * (step + 1) * torch.arange(g.numel(), dtype=torch.float32).view(shape)
                assert torch.equal(g, ref)
