"""Interleaved A/B of library variants in ONE process (cdna_hip_programming.md §5.4 rule 24):
each build_var/*/libprotoseg_hip.so is loaded side by side with the main library (RTLD_LOCAL),
and every rep times each library's call back to back, so clock / thermal drift hits all
variants alike. usage: python tools/ab_libs.py --protos 361 --call bwd_full [--reps 40]"""
import argparse
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))

import torch  # noqa: E402

from protoseg_amd import _lib  # noqa: E402

CSRC = os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd", "csrc")


def load(path):
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--protos", type=int, default=361)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--fmap", type=int, default=65)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--main-bwd", default="", help="backward kernels (protoseg_set_backward_kernel) to run the main library with")
    ap.add_argument("--call", default="bwd_full", choices=["bwd_full", "bwd_full_xsig", "fwd", "fwd_xsig", "push", "mask", "kld", "kldb", "kldc",
                                                       "bwdk"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    B, C, h, w, P, K = args.batch, 64, args.fmap, args.fmap, args.protos, 19
    gen = torch.Generator().manual_seed(0)
    x = torch.sigmoid(2 * torch.randn(B, C, h, w, generator=gen)).to(dev)
    protos = torch.rand(P, C, generator=gen).to(dev)
    wl = (torch.rand(K, P, generator=gen) - 0.5).to(dev)
    gl = torch.randn(B, h, w, K, generator=gen).to(dev)
    dist = torch.empty(B, P, h, w, device=dev)
    logits = torch.empty(B, h, w, K, device=dev)
    gx, gp, gw = torch.empty_like(x), torch.empty(P, C, device=dev), torch.empty(K, P, device=dev)
    libs = {"main": load(os.path.join(CSRC, "libprotoseg_hip.so"))}
    # backward kernel per library: --main-bwd for main (several: main@k1, main@k2 entries), a BWD file
    # in a variant's directory for that variant (else the process environment)
    bwd_of = {}
    if args.main_bwd:
        main = libs.pop("main")
        for k in args.main_bwd.split(","):
            libs[f"main@{k}"] = main
            bwd_of[f"main@{k}"] = k
    for d in sorted(glob.glob(os.path.join(CSRC, "build_var", "*", "libprotoseg_hip.so"))):
        name = os.path.basename(os.path.dirname(d))
        libs[name] = load(d)
        f = os.path.join(os.path.dirname(d), "BWD")
        if os.path.exists(f):
            bwd_of[name] = open(f).read().strip()
    first = next(iter(libs.values()))
    ws_b = max(lb.protoseg_l2_bwd_workspace_size(B, C, h, w, P, K) for lb in libs.values())
    ws = torch.empty(ws_b, device=dev, dtype=torch.uint8)
    P_, s = _lib.ptr, _lib.stream_of(dev)
    act = _lib.X_SIGMOID if args.call.endswith("xsig") else 0
    prec = _lib.PRECISIONS["bf16x3"]

    if args.call in ("push", "mask"):  # push argmin over 8 Cityscapes-sized maps (bench.py's push leg)
        n_img, ph, pw = 8, 129, 257
        xp = torch.sigmoid(2 * torch.randn(n_img, C, ph, pw, generator=gen)).to(dev)
        lab = torch.randint(0, K + 1, (n_img, 1024, 2048), generator=gen, dtype=torch.uint8).to(dev)
        mask = torch.empty((n_img, ph * pw), device=dev, dtype=torch.int32)
        pcls = torch.clamp(torch.arange(P) // max(1, P // K), max=K - 1).to(torch.int32).to(dev)
        keys = torch.empty((n_img, P), device=dev, dtype=torch.int64)
        second = torch.empty_like(keys)
        st = first.protoseg_patch_class_mask(P_(lab), _lib.U8, n_img, 1024, 2048, ph, pw, None, 0, P_(mask), s)
        assert st == 0

    if args.call in ("kld", "kldb", "kldc", "bwdk"):  # KLD forward (kldb: + backward, kldc: + compact backward) on the layer's distances (bench.py setup_kld: 8x8 label blocks)
        blocks = torch.randint(0, K + 1, (B, (h + 7) // 8, (w + 7) // 8), generator=gen)
        tgt = blocks.repeat_interleave(8, 1).repeat_interleave(8, 2)[:, :h, :w].reshape(B, -1).contiguous().to(dev)
        pcls = torch.clamp(torch.arange(P) // (P // K), max=K - 1).to(torch.int32).to(dev)
        mpc = int(torch.bincount(pcls.cpu().long()).max())
        kws_b = max(lb.protoseg_kld_workspace_size(B, P, h * w, K) for lb in libs.values())
        kws = torch.empty(kws_b, device=dev, dtype=torch.uint8)
        kloss = torch.empty((), device=dev)
        kg = torch.full((), 0.25, device=dev)
        gdist = torch.empty_like(dist)
        gcls = torch.empty(B * h * w, mpc, device=dev)
        pixc = torch.empty(B * h * w, device=dev, dtype=torch.int32)
        pslot = torch.empty(P, device=dev, dtype=torch.int32)
        st = first.protoseg_l2_fwd(P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0,
                                          _lib.PRECISIONS["bf16x3"], P_(dist), None, P_(logits), s)
        assert st == 0
        if args.call == "bwdk":  # the layer backward with the compact KLD gradient (protoseg_l2_bwd_kld)
            st = first.protoseg_kld_forward(P_(dist), B, P, h * w, P_(tgt), _lib.I64, P_(pcls), K, mpc,
                                                   P_(kloss), None, P_(kws), kws_b, s)
            st = st or first.protoseg_kld_backward_compact(P_(dist), B, P, h * w, P_(tgt), _lib.I64, P_(pcls),
                                                                  K, mpc, P_(kg), P_(kws), kws_b, P_(gcls), P_(pixc),
                                                                  P_(pslot), s)
            assert st == 0

    def call(lib, name=None):
        if name in bwd_of:
            if hasattr(lib, "protoseg_set_backward_kernel"):
                lib.protoseg_set_backward_kernel(bwd_of[name].encode())
        if args.call == "mask":
            st = lib.protoseg_patch_class_mask(P_(lab), _lib.U8, n_img, 1024, 2048, ph, pw, None, 0, P_(mask), s)
        elif args.call in ("kld", "kldb", "kldc"):
            st = lib.protoseg_kld_forward(P_(dist), B, P, h * w, P_(tgt), _lib.I64, P_(pcls), K, mpc, P_(kloss), None,
                                          P_(kws), kws_b, s)
            if args.call == "kldb" and st == 0:
                st = lib.protoseg_kld_backward(P_(dist), B, P, h * w, P_(tgt), _lib.I64, P_(pcls), K, mpc, P_(kg),
                                               P_(kws), kws_b, P_(gdist), s)
            if args.call == "kldc" and st == 0:
                st = lib.protoseg_kld_backward_compact(P_(dist), B, P, h * w, P_(tgt), _lib.I64, P_(pcls), K, mpc,
                                                       P_(kg), P_(kws), kws_b, P_(gcls), P_(pixc), P_(pslot), s)
        elif args.call == "bwdk":
            st = lib.protoseg_l2_bwd_kld(P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0, prec, P_(gl),
                                         P_(gcls), P_(pixc), P_(pslot), mpc, P_(gx), P_(gp), P_(gw), P_(ws), ws_b, s)
        elif args.call == "push":
            st = lib.protoseg_push_argmin(P_(xp), n_img, C, ph, pw, P_(protos), P, P_(pcls), P_(mask), P_(keys),
                                          P_(second), s)
        elif args.call.startswith("bwd"):
            st = lib.protoseg_l2_bwd(P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, act, prec, P_(gl), None,
                                     P_(gx), P_(gp), P_(gw), P_(ws), ws_b, s)
        else:
            st = lib.protoseg_l2_fwd(P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, act, prec, P_(dist), None,
                                     P_(logits), s)
        assert st == 0, lib.protoseg_last_error()

    ref = None
    for name, lib in libs.items():  # warm-up + the variants agree with main
        call(lib, name)
        torch.cuda.synchronize()
        out = (gdist if args.call == "kldb" else gcls if args.call == "kldc" else mask.float() if args.call == "mask" else
               kloss.reshape(1) if args.call == "kld" else keys.float() if args.call == "push" else
               torch.cat([gx.flatten(), gp.flatten(), gw.flatten()]) if args.call.startswith("bwd") else logits).clone()
        if ref is None:
            ref = out
        else:
            err = (out - ref).abs().max().item() / (ref.abs().max().item() + 1e-30)
            print(f"{name}: rel diff vs main {err:.2e}")
    times = {k: [] for k in libs}
    for _ in range(args.reps):
        for name, lib in libs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            call(lib, name)
            b.record()
            times[name].append((a, b))
    torch.cuda.synchronize()
    print(f"== {args.call} P={P} B={B} fmap={args.fmap}")
    for k, evs in times.items():
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        print(f"{k:14s} median {ms[len(ms) // 2] * 1e3:8.1f} us  min {ms[0] * 1e3:8.1f} us")
    # diagnostic builds (WAVE_STAMP): the last launch's per-phase s_memtime cycles, mean over waves
    for k, lib in libs.items():
        fn = getattr(lib, "protoseg_dev_wave_stamps", None)
        if fn is None:
            continue
        buf = (ctypes.c_ulonglong * (1024 * 16))()
        fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
        call(lib, k)
        torch.cuda.synchronize()
        assert fn(ctypes.addressof(buf), 1024 * 16) == 0
        rows = [list(buf[i * 16:(i + 1) * 16]) for i in range(1024)]
        rows = [r for r in rows if r[15] != 0]
        names = ["dma", "front0", "A0", "A1", "A2", "B0", "B1", "B2", "gxlast", "part", "wait+bar", "reduce",
                 "convert", "bar2", "prologue", "slab"]
        tot = sum(sum(r) for r in rows) / len(rows)
        print(f"{k}: stamps over {len(rows)} waves, total {tot:.0f} cyc/wave")
        for i, n in enumerate(names):
            v = sum(r[i] for r in rows) / len(rows)
            print(f"   {n:9s} {v:9.0f} cyc  {100 * v / tot:5.1f}%")


if __name__ == "__main__":
    main()
