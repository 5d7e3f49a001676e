"""Shared helpers for the GPU parity tests (import only inside -m gpu tests)."""
import numpy as np
import torch

from regcn_amd import graph as G

C = 0.01
TOL = 1e-4  # |delta| <= 1e-4 * max(1, |ref|)  (SURVEY.md §8(a) parity tolerances)


def rel_err(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float((np.abs(a - b) / np.maximum(1.0, np.abs(b))).max()) if a.size else 0.0


def assert_close(a, b, tol=TOL, what=""):
    e = rel_err(a, b)
    assert e <= tol, "%s max scaled error %.3g > %.3g" % (what, e, tol)


MODEL_CASES = {
    "uvrgcn_roth": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False),
    "uvrgcn_roth_ln": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=True),
    "lgcn_roth": dict(encoder_name="lgcn", decoder_name="roth", layer_norm=False),
    "lgcn_roth_ln": dict(encoder_name="lgcn", decoder_name="roth", layer_norm=True),
    "uvrgcn_murp_nores": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="murp", layer_norm=False,
                              use_residual_evolution=False),
    "uvrgcn_atth_beta": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="atth", layer_norm=True,
                             radius_anchor_beta=0.5),
    "lgcn_roth_bias_crel": dict(encoder_name="lgcn", decoder_name="roth", layer_norm=False,
                                use_entity_euclidean_bias=True, use_relation_specific_curvature=True),
    "uvrgcn_convtranse": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="hyperbolic_convtranse",
                              layer_norm=True),
    # d = 200 at the dataset shapes (tools/goldens/make_golden.py LARGE_CASES): ICEWS18's
    # R2 = 512 with hub rows over the inline budget, |E| = 80k snapshots (large-graph work
    # lists), GDELT's history length 7 for both encoders; their goldens hold the last
    # history embedding only ("embs_last")
    "uvrgcn_roth_r512_d200": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False),
    "uvrgcn_roth_e80k_d200": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False),
    "uvrgcn_roth_h7_d200": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False),
    "lgcn_roth_h7_d200": dict(encoder_name="lgcn", decoder_name="roth", layer_norm=True),
}


def build_hyperbolic_model(z, tag, device):
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    V, R, d, T = (int(v) for v in z["meta"])
    kw = dict(num_ents=V, num_rels=R, num_static_rels=0, num_words=0, h_dim=d, opn="sub", sequence_len=T,
              num_bases=d // 2, num_hidden_layers=2, dropout=0.2, c=C, self_loop=True, skip_connect=False,
              input_dropout=0.2, hidden_dropout=0.2, feat_dropout=0.2, entity_prediction=True,
              relation_prediction=True, use_cuda=True, gpu=0, radius_target=z["radius_target"],
              radius_msg_gamma=0.15)
    kw.update(MODEL_CASES[tag])
    m = HyperbolicRecurrentRGCN(**kw)
    sd = {k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd_")}
    m.load_state_dict(sd, strict=True)
    m = m.to(device).eval()
    glist = [G.build_sub_graph(V, R, z["snap%d" % t], True, device) for t in range(T)]
    return m, glist, (V, R, d, T)
