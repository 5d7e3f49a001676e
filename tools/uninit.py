"""Debug: does a training step read memory no kernel wrote?  With
torch.utils.deterministic.fill_uninitialized_memory every torch.empty is NaN-filled, so a
read of an unwritten element surfaces as a NaN loss or gradient.  Runs one get_loss_batches
+ backward of the CLI test model (lgcn / uvrgcn + RotH, d = 64) and reports non-finite
losses and gradients, then the library calls whose float outputs hold NaN.

  python tools/uninit.py [--encoder lgcn] [--d 64]
"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--encoder", default="lgcn")
    ap.add_argument("--decoder", default="roth")
    ap.add_argument("--d", type=int, default=64)
    a = ap.parse_args()
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = True
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    from regcn_amd.synthetic import CONFIGS, snapshot_series
    cfg = CONFIGS["icews14s_lgcn_roth"]
    V, R, T, per = cfg["V"], cfg["R"], cfg["T"], cfg["per_snap"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rt = np.random.default_rng(0).uniform(0.5, 3.0, V).astype(np.float32)
    m = HyperbolicRecurrentRGCN(a.decoder, a.encoder, V, R, 0, 0, a.d, "sub", T, num_bases=a.d // 2,
                                num_hidden_layers=2, dropout=0.0, c=0.01, self_loop=True, layer_norm=False,
                                input_dropout=0.0, hidden_dropout=0.0, feat_dropout=0.0, entity_prediction=True,
                                relation_prediction=True, use_cuda=True, gpu=0, radius_target=rt,
                                radius_msg_gamma=0.15).to(dev).train()
    snaps = snapshot_series(1, V, R, T + 1, per)
    glist = [G.build_sub_graph(V, R, s, True, dev) for s in snaps[:T]]
    tr = torch.from_numpy(snaps[T]).to(dev)
    # report the library calls whose float tensors contain NaN right after the call
    from regcn_amd import _lib
    real_call = _lib.call
    seen = []

    def checked(name, *args):
        rc = real_call(name, *args)
        torch.cuda.synchronize()
        seen.append(name)
        return rc

    _lib.call = checked
    try:
        with torch.autograd.detect_anomaly(check_nan=True):
            parts = m.get_loss_batches(glist, tr, None, True, 64,
                                       combine=lambda le, lr, ls, lrad: 0.7 * le + 0.3 * lr + ls.sum() + lrad)
    except RuntimeError as e:
        print("anomaly:", str(e)[:600], flush=True)
        parts = []
    torch.cuda.synchronize()
    _lib.call = real_call
    bad_l = [i for i, p in enumerate(parts) if not all(bool(torch.isfinite(t).all()) for t in p)]
    bad_g = [n for n, p in m.named_parameters() if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
    print("encoder %s decoder %s d %d: non-finite mini-batch losses %s; non-finite grads %s" % (
        a.encoder, a.decoder, a.d, bad_l, bad_g), flush=True)
    print("library calls:", sorted(set(seen)), flush=True)


if __name__ == "__main__":
    main()
