"""Parity of the HIP evaluation counts (eval_valid.py:159-197) with the oracle.

Counts are integers and must match exactly, except for pixels whose top-2 upsampled logits
(or distances) lie within 1e-5 of each other: there the f32 bilinear evaluation order of the
kernel, torch-CPU and the reference's CUDA may legitimately pick different indices. The tests
compute those near-tie pixels from a float64 upsample and allow at most that many differences.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import eval_oracle as eo

pytestmark = pytest.mark.gpu


def _evaluate():
    from protoseg_amd import evaluate
    return evaluate


def _case(B, h, w, H, W, K, P, seed):
    gen = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, h, w, K, generator=gen) * 3
    dist = torch.rand(B, P, h, w, generator=gen) * 20
    rng = np.random.default_rng(seed)
    blocks = rng.integers(0, K + 1, size=(B, (H + 7) // 8, (W + 7) // 8))
    anns = np.repeat(np.repeat(blocks, 8, 1), 8, 2)[:, :H, :W].astype(np.int64)
    pc = (np.arange(P) * K // P).astype(np.int32)
    return logits, dist, anns, pc


def _near_ties(t_bhwc_or_bchw, size, largest):
    up = F.interpolate(t_bhwc_or_bchw.double(), size=size, mode="bilinear", align_corners=False)
    v = torch.topk(up if largest else -up, 2, dim=1).values
    return int(((v[:, 0] - v[:, 1]).abs() < 1e-5).sum())


@pytest.mark.parametrize("B,h,w,H,W,K,P", [
    (2, 9, 17, 72, 135, 19, 38),       # non-integer scales
    (1, 17, 33, 129, 257, 5, 10),      # non-integer, few classes
    (2, 5, 7, 5, 7, 3, 6),             # identity size
    (1, 13, 13, 100, 100, 21, 42),     # pascal-like 21 classes
])
def test_eval_counts_match_oracle(device, B, h, w, H, W, K, P):
    ev = _evaluate()
    logits, dist, anns, pc = _case(B, h, w, H, W, K, P, seed=h * W + K)
    ref = eo.eval_counts(logits, anns, K, dist, pc)
    counts = torch.zeros(2 + 2 * K + P, dtype=torch.int64, device=device)
    ev.eval_counts(logits.to(device), torch.from_numpy(anns).to(device), counts, dist.to(device),
                   torch.from_numpy(pc).to(device))
    c = counts.cpu().numpy()
    tie_l = _near_ties(logits.permute(0, 3, 1, 2), (H, W), True)
    tie_d = _near_ties(dist, (H, W), False)
    assert abs(int(c[0]) - int(ref["correct"])) <= tie_l
    assert int(c[1]) == int(ref["total"])
    assert np.abs(c[2:2 + K] - ref["I"]).sum() <= tie_l
    assert np.abs(c[2 + K:2 + 2 * K] - ref["U"]).sum() <= 2 * tie_l
    assert np.abs(c[2 + 2 * K:] - ref["proto_counts"]).sum() <= 2 * (tie_l + tie_d)
    assert int(c[0]) == int(c[2:2 + K].sum())          # correct = sum of intersections
    assert np.all(c[2 + K:2 + 2 * K] >= c[2:2 + K])    # union >= intersection


def test_evaluator_accumulates_and_matches_metrics(device):
    ev = _evaluate()
    K, P = 19, 190
    logits, dist, anns, pc = _case(2, 17, 33, 129, 257, K, P, seed=7)
    e = ev.SegmentationEvaluator(K, torch.from_numpy(pc), device)
    for i in range(2):  # batches of one image accumulate like the reference's Counters
        e.update(logits[i:i + 1].to(device), torch.from_numpy(anns[i:i + 1]).to(device), dist[i:i + 1].to(device))
    r = e.result()
    ref = eo.eval_counts(logits, anns, K, dist, pc)
    acc, miou, _ = eo.metrics(int(ref["correct"]), int(ref["total"]), ref["I"], ref["U"])
    assert abs(r["pixel_accuracy"] - acc) < 0.05 and abs(r["mean_iou"] - miou) < 0.2   # north_star: mIoU +-0.2


def test_eval_lut_and_dtypes(device):
    """Raw Cityscapes ids through the CLS_CONVERT table (eval_valid.py:139) == converted labels."""
    from oracle import push_oracle as pu
    ev = _evaluate()
    K = 19
    logits, _, _, _ = _case(1, 9, 17, 72, 135, K, 19, seed=3)
    raw = np.random.default_rng(4).integers(0, 34, size=(1, 72, 135))
    lut = np.zeros(34, np.int32)
    for k, v in pu.CITYSCAPES_19_EVAL_CATEGORIES.items():
        lut[k] = v
    conv = lut[raw]
    outs = []
    for ann, tab in ((torch.from_numpy(conv).to(torch.uint8), None), (torch.from_numpy(raw).to(torch.int32),
                                                                       torch.from_numpy(lut))):
        c = torch.zeros(2 + 2 * K, dtype=torch.int64, device=device)
        ev.eval_counts(logits.to(device), ann.to(device), c, lut=None if tab is None else tab.to(device))
        outs.append(c.cpu())
    assert torch.equal(outs[0], outs[1])


def test_eval_full_resolution_properties(device):
    """Cityscapes eval shape: 129x257 maps upsampled to 1024x2048 (eval_valid.py:171-172): the
    class counts against the oracle (logits only; the oracle's [190, 1024, 2048] distance upsample
    is left to the small cases), plus the count invariants with distances."""
    ev = _evaluate()
    K, P = 19, 190
    logits, dist, anns, pc = _case(1, 129, 257, 1024, 2048, K, P, seed=11)
    counts = torch.zeros(2 + 2 * K + P, dtype=torch.int64, device=device)
    ev.eval_counts(logits.to(device), torch.from_numpy(anns).to(device), counts, dist.to(device),
                   torch.from_numpy(pc).to(device))
    c = counts.cpu().numpy()
    assert int(c[1]) == int((anns != 0).sum())
    assert int(c[0]) == int(c[2:2 + K].sum())
    assert 0 < int(c[2 + 2 * K:].sum()) <= 1024 * 2048
    ref = eo.eval_counts(logits, anns, K)
    tie_l = _near_ties(logits.permute(0, 3, 1, 2), (1024, 2048), True)
    assert abs(int(c[0]) - int(ref["correct"])) <= tie_l
    assert np.abs(c[2:2 + K] - ref["I"]).sum() <= tie_l
    assert np.abs(c[2 + K:2 + 2 * K] - ref["U"]).sum() <= 2 * tie_l
