"""One operand prep per training step (protoseg_l2_fwd_ex / protoseg_l2_bwd_ex / _kld_ex): the
forward's prep launch also writes the training backward's operand images (the standard image
block the wave-owned and fused kernels read) into a
caller buffer, and the backward
reads them instead of preparing its own. Same prep arithmetic, so every output is bit-identical
to the plain calls; the autograd path (prototype_layer) passes the buffer through ctx."""
import pytest
import torch

from oracle import protoseg_oracle as po

pytestmark = pytest.mark.gpu


def _ops():
    from protoseg_amd import _lib, ops
    return _lib, ops


def _inputs(device, B, h, w, P, K, seed):
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=seed)
    gen = torch.Generator().manual_seed(seed + 1)
    w_last = w_last + 0.05 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    g_dist = 0.01 * torch.randn(B, P, h, w, generator=gen)
    return [t.to(device) for t in (x, protos, w_last, g_logits, g_dist)]


@pytest.mark.parametrize("P,K,bwd,kind", [
    (361, 19, None, "fused"),        # the metric's 19 prototypes/class: the wave-owned backward
    (190, 19, None, "fused"),        # 10 prototypes/class                 reads the standard block
    (96, 32, None, "fused"),
    (190, 19, "wave", "fused"),
    (570, 19, None, "none"),         # two prototype chunks: no operands, plain calls
])
@pytest.mark.parametrize("activation", ["log", "linear"])
def test_fwd_bwd_with_operands_bit_identical(device, bwd_kernel, P, K, bwd, kind, activation):
    _lib, ops = _ops()
    if bwd:
        bwd_kernel(bwd)
    B, h, w = 2, 33, 31
    x, protos, w_last, g_logits, g_dist = _inputs(device, B, h, w, P, K, seed=P + K)
    act, prec = ops.ACT_KINDS[activation], ops.PRECISIONS["bf16x3"]
    nbytes = ops.train_operands_bytes(64, P, K, prec)
    assert (nbytes > 0) == (kind != "none")
    d0, l0, a0, o0 = ops.l2_forward(x, protos, w_last, 1e-4, act, prec, True, True, True)
    d1, l1, a1, o1 = ops.l2_forward(x, protos, w_last, 1e-4, act, prec, True, True, True, True)
    assert o0.numel() == 0 and o1.numel() == nbytes
    for a, b in ((d0, d1), (l0, l1), (a0, a1)):
        assert torch.equal(a, b)
    ref = ops.l2_backward(x, protos, w_last, g_logits, g_dist, 1e-4, act, prec, True, True, True)
    got = ops.l2_backward(x, protos, w_last, g_logits, g_dist, 1e-4, act, prec, True, True, True, o1)
    torch.cuda.synchronize()
    for name, a, b in zip(("g_x", "g_protos", "g_w"), ref, got):
        assert torch.equal(a, b), name


def test_operands_only_forward_and_x_sigmoid(device):
    """Every output NULL fills the operands only; the X_SIGMOID backward reads them too."""
    _lib, ops = _ops()
    B, h, w, P, K = 1, 29, 37, 361, 19
    x, protos, w_last, g_logits, _ = _inputs(device, B, h, w, P, K, seed=5)
    prec = ops.PRECISIONS["bf16x3"]
    act = _lib.ACT_LOG | _lib.X_SIGMOID
    _, _, _, ob = ops.l2_forward(x, protos, w_last, 1e-4, act, prec, False, False, False, True)
    assert ob.numel() == ops.train_operands_bytes(64, P, K, prec)
    ref = ops.l2_backward(x, protos, w_last, g_logits, None, 1e-4, act, prec, True, True, True)
    got = ops.l2_backward(x, protos, w_last, g_logits, None, 1e-4, act, prec, True, True, True, ob)
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_kld_backward_reads_operands(device):
    _lib, ops = _ops()
    B, h, w, P, K, mpc = 2, 17, 19, 361, 19, 19
    x, protos, w_last, g_logits, _ = _inputs(device, B, h, w, P, K, seed=9)
    prec = ops.PRECISIONS["bf16x3"]
    gen = torch.Generator().manual_seed(4)
    npix = B * h * w
    g_cls = torch.randn(npix, mpc, generator=gen).to(device)
    pix_cls = torch.randint(-1, K, (npix,), generator=gen, dtype=torch.int32).to(device)
    proto_slot = torch.tensor([(p // mpc) * 256 + p % mpc for p in range(P)], dtype=torch.int32, device=device)
    _, _, _, ob = ops.l2_forward(x, protos, w_last, 1e-4, 0, prec, True, True, False, True)
    ref = ops.l2_backward_kld(x, protos, w_last, g_logits, g_cls, pix_cls, proto_slot, mpc, 1e-4, 0, prec,
                              True, True, True)
    got = ops.l2_backward_kld(x, protos, w_last, g_logits, g_cls, pix_cls, proto_slot, mpc, 1e-4, 0, prec,
                              True, True, True, ob)
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_short_operands_buffer_fails_loudly(device):
    _lib, ops = _ops()
    x, protos, w_last, g_logits, _ = _inputs(device, 1, 9, 9, 361, 19, seed=2)
    prec = ops.PRECISIONS["bf16x3"]
    n = ops.train_operands_bytes(64, 361, 19, prec)
    short = torch.empty(n - 256, device=device, dtype=torch.uint8)
    d = torch.empty(1, 361, 9, 9, device=device)
    with pytest.raises(_lib.ProtosegError, match="operands"):
        _lib.call("protoseg_l2_fwd_ex", _lib.ptr(x), _lib.F32, 1, 64, 9, 9, _lib.ptr(protos), 361, _lib.ptr(w_last),
                  19, 1e-4, 0, prec, _lib.ptr(d), None, None, _lib.ptr(short), short.numel(), _lib.stream_of(device))


@pytest.mark.parametrize("P", [190, 361])
def test_autograd_layer_uses_forward_operands(device, P):
    """prototype_layer in a training graph: gradients equal l2_backward's without operands."""
    _lib, ops = _ops()
    B, h, w, K = 2, 21, 23, 19
    x, protos, w_last, g_logits, g_dist = _inputs(device, B, h, w, P, K, seed=P)
    xr, pr, wr = (t.clone().requires_grad_(True) for t in (x, protos, w_last))
    dist, logits, _ = ops.prototype_layer(xr, pr[:, :, None, None], wr)
    (logits * g_logits).sum().backward(retain_graph=True)
    ref = ops.l2_backward(x, protos, w_last, g_logits, None, 1e-4, 0, ops.PRECISIONS["bf16x3"], True, True, True)
    torch.cuda.synchronize()
    assert torch.equal(xr.grad, ref[0]) and torch.equal(pr.grad.reshape(P, 64), ref[1])
    assert torch.equal(wr.grad, ref[2])
    # a second backward over the retained graph reads the same operands again
    for t in (xr, pr, wr):
        t.grad = None
    ((logits * g_logits).sum() + (dist * g_dist).sum()).backward()
    ref2 = ops.l2_backward(x, protos, w_last, g_logits, g_dist, 1e-4, 0, ops.PRECISIONS["bf16x3"], True, True, True)
    torch.cuda.synchronize()
    assert torch.equal(xr.grad, ref2[0]) and torch.equal(pr.grad.reshape(P, 64), ref2[1])
    assert torch.equal(wr.grad, ref2[2])


def _fwd_operands(_lib, x, protos, w_last, act, prec, buf, ready=False):
    B, C, H, W = x.shape
    P, K = protos.shape[0], w_last.shape[0]
    d = torch.empty(B, P, H, W, device=x.device)
    lg = torch.empty(B, H, W, K, device=x.device)
    _lib.call("protoseg_l2_fwd_ex", _lib.ptr(x), _lib.F32, B, C, H, W, _lib.ptr(protos), P, _lib.ptr(w_last), K,
              1e-4, act | (_lib.OPERANDS_READY if ready else 0), prec, _lib.ptr(d), None, _lib.ptr(lg),
              _lib.ptr(buf), buf.numel(), _lib.stream_of(x.device))
    return d, lg


@pytest.mark.parametrize("P,K", [(361, 19), (190, 19), (100, 7), (96, 32)])
@pytest.mark.parametrize("activation", ["log", "linear"])
def test_adam_prep_equals_adam_then_prep(device, P, K, activation):
    """protoseg_l2_adam_prep (Adam.layer_step_with_operands) = protoseg_adam_step of both tensors
    (per-group lr / weight decay) followed by the forward's prep of the updated values, bit for
    bit: parameters, moments, step counts and every byte of the operand block; a forward with
    PROTOSEG_OPERANDS_READY on that block equals the forward that builds its own."""
    _lib, ops = _ops()
    from protoseg_amd.optim import Adam
    prec, act = ops.PRECISIONS["bf16x3"], ops.ACT_KINDS[activation]
    assert _lib.load().protoseg_l2_adam_prep_supported(64, P, K, prec)
    x, protos, w_last, _, _ = _inputs(device, 2, 13, 11, P, K, seed=3 * P + K)
    gen = torch.Generator().manual_seed(P + 17 * K)
    rnd = lambda *s: torch.randn(*s, generator=gen).to(device)  # noqa: E731
    g_p, g_w = 1e-2 * rnd(P, 64), 1e-2 * rnd(K, P)
    m0 = (1e-3 * rnd(P, 64), 1e-3 * rnd(K, P))
    v0 = (1e-5 * rnd(P, 64).abs(), 1e-5 * rnd(K, P).abs())
    nbytes = ops.train_operands_bytes(64, P, K, prec)
    runs = []
    for fused in (False, True):
        p = torch.nn.Parameter(protos.contiguous().clone())
        w = torch.nn.Parameter(w_last.contiguous().clone())  # (the identity init is a transpose)
        p.grad, w.grad = g_p.clone(), g_w.clone()
        opt = Adam([{"params": [p], "lr": 2.5e-3, "weight_decay": 0.0},
                    {"params": [w], "lr": 1e-3, "weight_decay": 5e-4}])
        for t, m, v in ((p, m0[0], v0[0]), (w, m0[1], v0[1])):
            opt.state[t] = {"exp_avg": m.clone(), "exp_avg_sq": v.clone(), "step": torch.tensor(4.0)}
        buf = torch.full((nbytes,), 0xAB, device=device, dtype=torch.uint8)
        for _ in range(2):  # two steps: the device step counts advance once per call
            if fused:
                assert opt.layer_step_with_operands(p, w, buf, 1e-4, act, prec)
            else:
                opt.step()
                _fwd_operands(_lib, x, p.detach(), w.detach(), act, prec, buf)
        torch.cuda.synchronize()
        runs.append((p.detach(), w.detach(), opt.state[p]["exp_avg"], opt.state[p]["exp_avg_sq"],
                     opt.state[w]["exp_avg"], opt.state[w]["exp_avg_sq"], opt._counter(p), opt._counter(w), buf))
    names = ("protos", "w_last", "m_p", "v_p", "m_w", "v_w", "step_p", "step_w", "operands")
    for name, a, b in zip(names, *runs):
        assert torch.equal(a, b), name
    assert int(runs[1][6][0]) == 6 and int(runs[1][7][0]) == 6
    p, w, buf = runs[1][0], runs[1][1], runs[1][8]
    ref = _fwd_operands(_lib, x, p, w, act, prec, torch.empty(nbytes, device=device, dtype=torch.uint8))
    got = _fwd_operands(_lib, x, p, w, act, prec, buf, ready=True)
    torch.cuda.synchronize()
    assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])


def test_adam_prep_with_other_groups_steps_each_tensor_once(device):
    """An optimizer that also holds other groups (the reference's one joint Adam over backbone,
    add-on, prototypes and last layer, module.py:391): layer_step_with_operands then step() updates
    every tensor exactly once per iteration, the same bits and step counts as step() alone."""
    _lib, ops = _ops()
    from protoseg_amd.optim import Adam
    prec, act = ops.PRECISIONS["bf16x3"], ops.ACT_KINDS["log"]
    P, K = 190, 19
    x, protos, w_last, _, _ = _inputs(device, 1, 9, 9, P, K, seed=11)
    gen = torch.Generator().manual_seed(12)
    rnd = lambda *s: torch.randn(*s, generator=gen).to(device)  # noqa: E731
    grads = (1e-2 * rnd(P, 64), 1e-2 * rnd(K, P), 1e-2 * rnd(33, 7))
    other = rnd(33, 7)
    nbytes = ops.train_operands_bytes(64, P, K, prec)
    runs = []
    for fused in (False, True):
        p = torch.nn.Parameter(protos.contiguous().clone())
        w = torch.nn.Parameter(w_last.contiguous().clone())
        o = torch.nn.Parameter(other.clone())
        opt = Adam([{"params": [o], "lr": 1e-4, "weight_decay": 5e-4},
                    {"params": [p], "lr": 2.5e-3, "weight_decay": 0.0},
                    {"params": [w], "lr": 1e-3, "weight_decay": 5e-4}])
        buf = torch.empty((nbytes,), device=device, dtype=torch.uint8)
        for _ in range(3):
            p.grad, w.grad, o.grad = (g.clone() for g in grads)
            if fused:
                assert opt.layer_step_with_operands(p, w, buf, 1e-4, act, prec)
            opt.step()
        torch.cuda.synchronize()
        runs.append([t.detach().clone() for t in (p, w, o)] +
                    [opt.state[t][k].clone() for t in (p, w, o) for k in ("exp_avg", "exp_avg_sq")] +
                    [opt._counter(t).clone() for t in (p, w, o)])
    for i, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), i
    assert [int(c[0]) for c in runs[1][-3:]] == [3, 3, 3]


def test_operands_ready_tracks_parameter_writes(device):
    """Adam.operands_ready: True right after the fused update for the same block / eps / activation
    / precision, False after any other write to either parameter (push's in-place copy) or for
    another block or activation."""
    _lib, ops = _ops()
    from protoseg_amd.optim import Adam
    prec, act = ops.PRECISIONS["bf16x3"], ops.ACT_KINDS["log"]
    _, protos, w_last, _, _ = _inputs(device, 1, 9, 9, 190, 19, seed=13)
    p = torch.nn.Parameter(protos.contiguous().clone())
    w = torch.nn.Parameter(w_last.contiguous().clone())
    opt = Adam([p, w], lr=1e-3)
    buf = torch.empty((ops.train_operands_bytes(64, 190, 19, prec),), device=device, dtype=torch.uint8)
    assert not opt.operands_ready(p, w, buf, 1e-4, act, prec)
    p.grad, w.grad = torch.ones_like(p), torch.ones_like(w)
    assert opt.layer_step_with_operands(p, w, buf, 1e-4, act, prec)
    opt.step()
    assert opt.operands_ready(p, w, buf, 1e-4, act, prec)
    assert not opt.operands_ready(p, w, buf, 1e-4, ops.ACT_KINDS["linear"], prec)
    assert not opt.operands_ready(p, w, buf.clone(), 1e-4, act, prec)
    with torch.no_grad():
        p.copy_(p.detach().clone())  # push_prototypes' write of the projected prototypes
    assert not opt.operands_ready(p, w, buf, 1e-4, act, prec)
    p.grad, w.grad = torch.ones_like(p), torch.ones_like(w)
    assert opt.layer_step_with_operands(p, w, buf, 1e-4, act, prec)
    opt.step()
    assert opt.operands_ready(p, w, buf, 1e-4, act, prec)
    w.data = w.data[:, :150].contiguous()  # prune_prototypes' column selection (a new address)
    assert not opt.operands_ready(p, w, buf, 1e-4, act, prec)


def test_operands_ready_refused_without_a_served_block(device):
    _lib, ops = _ops()
    prec = ops.PRECISIONS["bf16x3"]
    x, protos, w_last, _, _ = _inputs(device, 1, 9, 9, 570, 19, seed=2)  # two chunks: no block
    assert not _lib.load().protoseg_l2_adam_prep_supported(64, 570, 19, prec)
    d = torch.empty(1, 570, 9, 9, device=device)
    with pytest.raises(_lib.ProtosegError, match="OPERANDS_READY"):
        _lib.call("protoseg_l2_fwd_ex", _lib.ptr(x), _lib.F32, 1, 64, 9, 9, _lib.ptr(protos), 570, _lib.ptr(w_last),
                  19, 1e-4, _lib.ACT_LOG | _lib.OPERANDS_READY, prec, _lib.ptr(d), None, None, None, 0,
                  _lib.stream_of(device))


@pytest.mark.parametrize("B,P", [(2, 361), (3, 190)])
def test_folded_layer_step_graph_matches_separate_launches(device, monkeypatch, B, P):
    """bench.py's layer step with the prep folded into the optimizer launch (forward with
    PROTOSEG_OPERANDS_READY reading the images the previous step's protoseg_l2_adam_prep wrote),
    eager and then replayed as one HIP graph, gives the parameters and moments of the same step
    run with Adam and the forward's prep as separate launches, bit for bit, over 6 steps."""
    import bench
    steps = {}
    for fold in ("1", "0"):
        monkeypatch.setenv("PROTOSEG_FOLD_PREP", fold)
        s = bench.LayerStep(B, 64, 17, 19, P, 19, torch.float32, device, bench.SEED)
        assert s.fold == (fold == "1")
        stream = torch.cuda.Stream(device)
        with torch.cuda.stream(stream):
            for _ in range(3):
                s.fwd(), s.bwd(), s.opt_step()
            torch.cuda.synchronize()
            g = bench.capture(lambda s=s: [s.fwd(), s.bwd(), s.opt_step()], stream)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
        steps[fold] = (s, g)  # the graph points into the step's buffers: keep both alive
    a, b = steps["1"][0], steps["0"][0]
    assert a.ops_ready and not b.ops_ready
    for name, x, y in (("protos", a.protos, b.protos), ("w_last", a.w_last, b.w_last),
                       ("logits", a.logits, b.logits), ("g_p", a.g_p, b.g_p)):
        assert torch.equal(x, y), name
    for pa, pb in zip(a.params, b.params):
        assert torch.equal(a.opt.state[pa]["exp_avg"], b.opt.state[pb]["exp_avg"])
        assert torch.equal(a.opt.state[pa]["exp_avg_sq"], b.opt.state[pb]["exp_avg_sq"])
        assert int(a.opt._counter(pa)[0]) == int(b.opt._counter(pb)[0]) == 6
