"""The CPU baseline's push loop (push.py:186, 214-230 verbatim: torch.LongTensor labels and one
.item() per pixel) builds the same class -> patch lists, in the same list(set) order, as the
numpy restatement the parity tests use."""
import numpy as np

from oracle import push_oracle as pu


def test_torch_item_loop_matches_numpy_restatement():
    rng = np.random.default_rng(5)
    for H, W, h, w in ((40, 47, 9, 11), (64, 128, 8, 16), (33, 20, 33, 20)):
        lab = rng.integers(0, 20, size=(H, W))
        a = pu.class_to_patch_index_dict(lab, h, w, 19)
        b = pu.class_to_patch_index_dict_torch(lab, h, w, 19)
        assert a.keys() == b.keys()
        for k in a:
            assert a[k] == b[k]
