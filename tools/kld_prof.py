"""Runs the KLD forward / backward (dense and compact) and the layer backward with each gradient
at the bench shape (B from $B, default 32, 65x65, K=19; P from $P, default 190) a few times, for rocprofv3
--kernel-trace --stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda:0")
st = bench.LayerStep(int(os.environ.get("B", 32)), 64, 65, 65, int(os.environ.get("P", 190)), 19, torch.float32, dev, bench.SEED)
st.setup_kld(bench.SEED)
st.fwd()
for _ in range(10):
    st.fwd()
    st.bwd()
    st.kld_fwd()
    st.kld_bwd()
    st.bwd_gd()
    st.kld_bwd_compact()
    st.bwd_kld()
torch.cuda.synchronize()
print("loss", float(st.kld_loss))
