"""Compact summary of a bench.py log's JSON line (headline, kernels, side lines)."""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
print("headline", d["value"], "img/s", d["ms_per_step"], "ms/step", "roofline", json.dumps(d["roofline"]))
print("kernels", json.dumps(d.get("kernels")))
for k in ("protos_190",):
    if k in d:
        print(k, d[k]["ms_per_step"], json.dumps(d[k]["kernels"]))
if "kld_step" in d:
    for p, v in d["kld_step"].items():
        print("kld", p, v["ms_per_step"], "ratio", v["ratio_to_plain_step"], "fwd", v["kld_forward_ms"], "bwd", v["kld_backward_ms"])
if "push" in d:
    p = d["push"]
    print("push", p["ms_per_img"], "argmin", p["argmin_kernel_ms_per_img"], "frac", p["roofline"]["frac"],
          "one", json.dumps(p.get("images_per_call_1")))
if "small_batch" in d:
    print("small", json.dumps({k: v["ms_per_step"] for k, v in d["small_batch"].items()}))
if "wide_family" in d:
    for k, v in d["wide_family"].items():
        print("wide", k, v["ms_per_step"], "fwd", v["fwd_ms"], v["roofline_fwd"]["frac"], "bwd", v["bwd_ms"], v["roofline_bwd"]["frac"])
for k in ("add_on_sigmoid", "train_step", "cpu_baseline", "eval", "knn_search"):
    if k in d:
        print(k, json.dumps(d[k])[:400])
