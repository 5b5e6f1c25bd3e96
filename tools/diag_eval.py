"""Diagnostics: where do eval negative logits differ between the HIP step and the oracle?"""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'tests'), os.path.join(os.path.dirname(__file__), '..', 'tgb-tgn-dgl_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np, torch
from parity_harness import Pair, rel_err
# cos accuracy: GPU vs CPU at wiki-scale arguments
x = (torch.rand(1_000_000) * 5.4e6 - 2.7e6).float()
gc = torch.cos(x.cuda()).cpu(); cc = torch.cos(x)
print("torch cos gpu-vs-cpu max abs diff", float((gc - cc).abs().max()))
p = Pair(N=400, E=1800, d=172, B=200, Kn_eval=20, seed=0)
for s in range(2):
    if s: p.sync_from_ref()
    r = p.train_step()
    print("train", s, rel_err(r["pos"], r["ref_pos"]), rel_err(r["neg"], r["ref_neg"]))
p.sync_from_ref()
r = p.eval_step(quirk=True)
d = np.abs(r["neg"] - r["ref_neg"])
print("eval pos", rel_err(r["pos"], r["ref_pos"]), "neg", rel_err(r["neg"], r["ref_neg"]), "mrr", r["mrr"], r["ref_mrr"])
idx = np.argsort(-d.ravel())[:10]
for k in idx:
    i, c = divmod(int(k), d.shape[1])
    print("row", i, c, r["neg"][i, c], r["ref_neg"][i, c], d[i, c])
print("quantiles", np.quantile(d, [0.5, 0.9, 0.99, 0.999, 1.0]))
r = p.eval_step(quirk=False)
print("noquirk eval neg vs ref(quirk) ", rel_err(r["neg"], r["ref_neg"]))
