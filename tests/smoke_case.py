"""One tiny hot-path invocation on a HIP device, checked against the CPU oracle
(used by __graft_entry__.smoke())."""
import numpy as np
import torch


def run_smoke(device):
    from oracle import graph as OG
    from oracle import model as OM
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN

    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    V, R, d, T = 300, 20, 200, 3
    snaps = [np.stack([rng.integers(0, V, 150), rng.integers(0, R, 150), rng.integers(0, V, 150)], 1)
             for _ in range(T + 1)]
    m = HyperbolicRecurrentRGCN("roth", "lgcn", V, R, 0, 0, d, "sub", T, num_bases=100, num_hidden_layers=2,
                                dropout=0.2, c=0.01, self_loop=True, entity_prediction=True,
                                relation_prediction=True, use_cuda=True, gpu=0, radius_msg_gamma=0.15)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(device).eval()
    glist = [G.build_sub_graph(V, R, s, True, device) for s in snaps[:T]]
    test = torch.from_numpy(snaps[T])
    _, score, score_rel = m.predict(glist, R, None, test.to(device), True)
    torch.cuda.synchronize()
    cfg = dict(c=0.01, n_layers=2, n_bases=100, radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
               radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True, encoder="lgcn",
               decoder="roth", layer_norm=False)
    _, ref, ref_rel, _, _ = OM.hyperbolic_predict(sd, cfg, [OG.build_sub_graph(V, R, s) for s in snaps[:T]], test)
    for got, want in ((score, ref), (score_rel, ref_rel)):
        err = ((got.cpu().double() - want.double()).abs() / want.double().abs().clamp(min=1.0)).max().item()
        assert err <= 1e-4, "smoke parity failed: %.3g" % err
    print("smoke ok: lgcn+roth predict on %s matches the oracle (V=%d, d=%d, T=%d)" % (device, V, d, T))
