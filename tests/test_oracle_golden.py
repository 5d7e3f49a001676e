"""Pin the CPU oracle against golden vectors produced by the reference itself
(tools/goldens/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import graph as og
from oracle import layers as ol
from oracle import model as om
from oracle import ops

C = 0.01


def close(a, b, tol=1e-4):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = np.abs(a - b) / np.maximum(1.0, np.abs(b))
    assert err.max() <= tol, err.max()


@pytest.mark.parametrize("tag", ["small", "mid", "empty_rel"])
def test_graph_indexing(golden, tag):
    z = golden("graph_indexing.npz")
    V, R = z[tag + "_meta"]
    g = og.build_sub_graph(int(V), int(R), z[tag + "_triples"])
    for k in ("src", "dst", "type", "in_deg", "uniq_r", "r_len"):
        np.testing.assert_array_equal(g[k], z[tag + "_" + k], err_msg=k)
    np.testing.assert_array_equal(g["norm"], z[tag + "_norm"])
    np.testing.assert_array_equal(g["enorm"], z[tag + "_enorm"])
    for a, b in g["r_len"]:
        assert set(g["r_to_e"][a:b].tolist()) == set(z[tag + "_r_to_e"][a:b].tolist())


@pytest.mark.parametrize("cname,c", [("c01", 0.01), ("c05", 0.05)])
def test_ops(golden, cname, c):
    z = golden("ops.npz")
    x, v, y, rad = (torch.from_numpy(z[cname + k]) for k in ("_x", "_v", "_y", "_rad"))
    close(ops.project(x, c), z[cname + "_project"])
    close(ops.log0(x, c), z[cname + "_log0"])
    close(ops.exp0(v, c), z[cname + "_exp0"])
    xb = ops.project(x, c)
    close(ops.mobius_add(xb, y, c), z[cname + "_mobius"])
    close(ops.hyperbolic_distance(xb, y, c), z[cname + "_dist"])
    close(ops.get_radius(x), z[cname + "_radius"])
    close(ops.apply_radius(y, rad, c), z[cname + "_apply_radius"])
    L = ops.to_lorentz(y, c)
    close(L, z[cname + "_to_lorentz"])
    close(ops.to_poincare(L, c), z[cname + "_to_poincare"])
    close(ops.lorentz_centroid(L, torch.from_numpy(z[cname + "_w"]), c), z[cname + "_centroid"])


def _graph(z, prefix=""):
    V, R = int(z[prefix + "meta"][0]), int(z[prefix + "meta"][1])
    return og.build_sub_graph(V, R, z[prefix + "triples"])


@pytest.mark.parametrize("gname,gamma", [("g0", 0.0), ("g15", 0.15)])
@pytest.mark.parametrize("skip", [False, True])
def test_union_layer(golden, gname, gamma, skip):
    z = golden("layer_union.npz")
    g = _graph(z)
    t = lambda k: torch.from_numpy(z[k])  # noqa: E731
    sk = (t("w_skip_weight"), t("w_skip_bias"), t("prev_h")) if skip else None
    y = ol.union_layer(g, t("h"), t("rel"), t("w_weight_neighbor"), t("w_loop_weight"),
                       t("w_evolve_loop_weight"), C, gamma, skip=sk)
    close(y, z["%s_%s_out" % (gname, "skip" if skip else "noskip")])


def test_euclid_layer(golden):
    z = golden("layer_euclid.npz")
    g = _graph(z)
    t = lambda k: torch.from_numpy(z[k])  # noqa: E731
    y = ol.euclid_union_layer(g, t("h"), t("rel"), t("w_weight_neighbor"), t("w_loop_weight"),
                              t("w_evolve_loop_weight"))
    close(y, z["out"])


@pytest.mark.parametrize("tag,skip", [("s2", False), ("s2", True), ("s4", False), ("s1", False),
                                      ("s20", False)])
def test_lorentz_layer(golden, tag, skip):
    z = golden("layer_lorentz.npz")
    g = _graph(z, tag + "_")
    t = lambda k: torch.from_numpy(z[tag + "_" + k])  # noqa: E731
    V, R, d, nb = (int(v) for v in z[tag + "_meta"])
    nb = min(nb, 2 * R)
    sk = (t("w_skip_weight"), t("w_skip_bias"), t("prev_h")) if skip else None
    y = ol.lorentz_layer(g, t("h"), t("rel"), t("w_weight"), t("w_loop_weight"),
                         t("w_evolve_loop_weight"), C, nb, skip=sk)
    close(y, z[tag + ("_skip" if skip else "_noskip") + "_out"])


MODEL_CASES = {
    "uvrgcn_roth": dict(encoder="hyperbolic_uvrgcn", decoder="roth", layer_norm=False),
    "uvrgcn_roth_ln": dict(encoder="hyperbolic_uvrgcn", decoder="roth", layer_norm=True),
    "lgcn_roth": dict(encoder="lgcn", decoder="roth", layer_norm=False),
    "lgcn_roth_ln": dict(encoder="lgcn", decoder="roth", layer_norm=True),
    "uvrgcn_murp_nores": dict(encoder="hyperbolic_uvrgcn", decoder="murp", layer_norm=False,
                              use_residual_evolution=False),
    "uvrgcn_atth_beta": dict(encoder="hyperbolic_uvrgcn", decoder="atth", layer_norm=True,
                             radius_anchor_beta=0.5),
    "lgcn_roth_bias_crel": dict(encoder="lgcn", decoder="roth", layer_norm=False),
    "uvrgcn_convtranse": dict(encoder="hyperbolic_uvrgcn", decoder="hyperbolic_convtranse",
                              layer_norm=True),
    "uvrgcn_roth_r512_d200": dict(encoder="hyperbolic_uvrgcn", decoder="roth", layer_norm=False),
    "uvrgcn_roth_e80k_d200": dict(encoder="hyperbolic_uvrgcn", decoder="roth", layer_norm=False),
    "uvrgcn_roth_h7_d200": dict(encoder="hyperbolic_uvrgcn", decoder="roth", layer_norm=False),
    "lgcn_roth_h7_d200": dict(encoder="lgcn", decoder="roth", layer_norm=True),
}


def model_cfg(tag, d):
    cfg = dict(c=C, n_layers=2, n_bases=d // 2, radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
               radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True)
    cfg.update(MODEL_CASES[tag])
    return cfg


def load_model_case(z):
    sd = {k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd_")}
    V, R, d, T = (int(v) for v in z["meta"])
    glist = [og.build_sub_graph(V, R, z["snap%d" % t]) for t in range(T)]
    return sd, glist, torch.from_numpy(z["test"]), (V, R, d, T)


@pytest.mark.parametrize("tag", list(MODEL_CASES))
def test_hyperbolic_model(golden, tag):
    z = golden("model_%s.npz" % tag)
    sd, glist, test, (V, R, d, T) = load_model_case(z)
    all_tr, score, score_rel, embs, h0 = om.hyperbolic_predict(sd, model_cfg(tag, d), glist, test)
    np.testing.assert_array_equal(all_tr.numpy(), z["all_triples"])
    if "embs" in z:
        close(torch.stack(embs), z["embs"])
    else:  # dataset-shaped goldens: the last history embedding
        close(embs[-1], z["embs_last"])
    close(h0, z["h0"])
    close(score, z["score"])
    close(score_rel, z["score_rel"])


@pytest.mark.parametrize("tag", ["noln", "ln", "ln_d200"])
def test_euclid_model(golden, tag):
    z = golden("rrgcn_%s.npz" % tag)
    sd, glist, test, (V, R, d, T) = load_model_case(z)
    cfg = dict(layer_norm=tag.startswith("ln"), n_layers=2)
    all_tr, score, score_rel, embs, h0 = om.euclid_predict(sd, cfg, glist, test)
    close(torch.stack(embs), z["embs"])
    close(h0, z["h0"])
    close(score, z["score"])
    close(score_rel, z["score_rel"])


def test_score_and_ce(golden):
    z = golden("score.npz")
    t = lambda k: torch.from_numpy(z[k])  # noqa: E731
    q, e, bias, scale, margin = t("q"), t("e"), t("bias"), t("scale"), t("margin")
    close(om.dist_score(q, e, None, C), z["score_plain"])
    close(om.dist_score(q, e, bias, C, scale, margin), z["score_bias"])
    close(om.dist_score(q, e, bias, C, scale, margin, t("c_r"), True), z["score_crel"])
    close(om.dist_score(q, e, None, C, scale, margin, None, True), z["score_dist"])
    close(om.ce_loss(q, e, t("target"), C, bias, scale, margin), z["ce_bias"])
    close(om.ce_loss(q, e, t("target"), C, bias, scale, margin, t("c_r"), True), z["ce_crel"])


def test_rank(golden):
    z = golden("rank.npz")
    V, R = (int(v) for v in z["meta"])
    tr = torch.from_numpy(z["all_triples"])
    ans_e = om.answers_for_filter(z["snap"], R, False)
    ans_r = om.answers_for_filter(z["snap"], R, True)
    mf, m, rank, frank = om.total_rank(tr, torch.from_numpy(z["score"]), ans_e)
    np.testing.assert_array_equal(rank.numpy(), z["rank"])
    np.testing.assert_array_equal(frank.numpy(), z["frank"])
    mfr, mr, rank_r, frank_r = om.total_rank(tr, torch.from_numpy(z["score_rel"]), ans_r, True)
    np.testing.assert_array_equal(rank_r.numpy(), z["rank_r"])
    np.testing.assert_array_equal(frank_r.numpy(), z["frank_r"])
    np.testing.assert_allclose([m, mf, mr, mfr], z["mrr"], rtol=1e-6)


TRAIN_CASES = {
    "uvrgcn_roth": dict(encoder="hyperbolic_uvrgcn", decoder="roth", layer_norm=False),
    "lgcn_roth": dict(encoder="lgcn", decoder="roth", layer_norm=False),
    "lgcn_roth_ln_skip": dict(encoder="lgcn", decoder="roth", layer_norm=True, skip_connect=True),
    "uvrgcn_murp_nores": dict(encoder="hyperbolic_uvrgcn", decoder="murp", layer_norm=False,
                              use_residual_evolution=False),
    "uvrgcn_atth_beta": dict(encoder="hyperbolic_uvrgcn", decoder="atth", layer_norm=True, radius_anchor_beta=0.5),
    "uvrgcn_convtranse": dict(encoder="hyperbolic_uvrgcn", decoder="hyperbolic_convtranse", layer_norm=True),
}


def train_cfg(tag, d):
    cfg = dict(c=C, n_layers=2, n_bases=d // 2, radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
               radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True)
    cfg.update(TRAIN_CASES[tag])
    return cfg


@pytest.mark.parametrize("tag", list(TRAIN_CASES))
def test_oracle_training_grads_vs_reference(golden, tag):
    """f1 pin: the oracle's get_loss + torch autograd reproduce the reference's loss values and
    every parameter gradient of one training mini-batch (tools/goldens/make_golden.py train)."""
    z = golden("train_%s.npz" % tag)
    V, R, d, T = (int(v) for v in z["meta"])
    sd = {k[3:]: torch.from_numpy(v).double() if v.dtype == np.float32 else torch.from_numpy(v)
          for k, v in z.items() if k.startswith("sd_")}
    for k in sd:
        if "grad_" + k in z:
            sd[k].requires_grad_(True)
    glist = [og.build_sub_graph(V, R, z["snap%d" % t]) for t in range(T)]
    le, lr, ls, lrad = om.hyperbolic_get_loss(sd, train_cfg(tag, d), glist, torch.from_numpy(z["batch"]),
                                              z["radius_target"])
    tw = float(z["task_weight"])
    loss = tw * le + (1 - tw) * lr + ls.sum() + lrad
    np.testing.assert_allclose([float(x.detach().sum()) for x in (le, lr, lrad, loss)], z["losses"][[0, 1, 3, 4]],
                               rtol=1e-5, atol=1e-6)
    loss.backward()
    n = 0
    for k in list(z):
        if k.startswith("grad_"):
            g = sd[k[5:]].grad
            ref = torch.from_numpy(z[k]).double()
            scale = max(1e-3, float(ref.abs().max()))
            err = float((g - ref).abs().max()) / scale
            assert err <= 1e-3, "%s: %.3g" % (k, err)
            n += 1
    assert n >= 20


@pytest.mark.parametrize("tag", ["noln", "ln"])
def test_oracle_euclid_training_grads_vs_reference(golden, tag):
    z = golden("train_rrgcn_%s.npz" % tag)
    V, R, d, T = (int(v) for v in z["meta"])
    sd = {k[3:]: torch.from_numpy(v).double() if v.dtype == np.float32 else torch.from_numpy(v)
          for k, v in z.items() if k.startswith("sd_")}
    for k in sd:
        if "grad_" + k in z:
            sd[k].requires_grad_(True)
    glist = [og.build_sub_graph(V, R, z["snap%d" % t]) for t in range(T)]
    le, lr, ls = om.euclid_get_loss(sd, dict(layer_norm=(tag == "ln"), n_layers=2), glist,
                                    torch.from_numpy(z["batch"]))
    tw = float(z["task_weight"])
    loss = tw * le + (1 - tw) * lr + ls.sum()
    np.testing.assert_allclose([float(x.detach().sum()) for x in (le, lr, loss)], z["losses"][[0, 1, 3]],
                               rtol=1e-5, atol=1e-6)
    loss.backward()
    n = 0
    for k in list(z):
        if k.startswith("grad_"):
            ref = torch.from_numpy(z[k]).double()
            err = float((sd[k[5:]].grad - ref).abs().max()) / max(1e-3, float(ref.abs().max()))
            assert err <= 1e-3, "%s: %.3g" % (k, err)
            n += 1
    assert n >= 15


ANALYSIS_CASES = {
    "uvrgcn_roth_beta": dict(encoder="hyperbolic_uvrgcn", decoder="roth", layer_norm=False, radius_anchor_beta=0.5),
    "lgcn_roth_ln": dict(encoder="lgcn", decoder="roth", layer_norm=True),
    "uvrgcn_murp_nores": dict(encoder="hyperbolic_uvrgcn", decoder="murp", layer_norm=False,
                              use_residual_evolution=False),
}
_BUFFERS = ("c", "radius_target")


@pytest.mark.parametrize("tag", list(ANALYSIS_CASES))
def test_oracle_analysis_vs_reference(golden, tag):
    """N1 pin (--run-analysis): the oracle's time gates, their means and the last radius-evolution
    stats of the eval forward, and the total gradient norm of one mini-batch (log_gradient_stats
    over the parameters that get a gradient) equal the reference's (analysis_*.npz)."""
    z = golden("analysis_%s.npz" % tag)
    V, R, d, T = (int(v) for v in z["meta"])
    cfg = dict(c=C, n_layers=2, n_bases=d // 2, radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
               radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True)
    cfg.update(ANALYSIS_CASES[tag])
    sd = {k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd_")}
    glist = [og.build_sub_graph(V, R, z["snap%d" % t]) for t in range(T)]
    ana = {}
    om.hyperbolic_forward(sd, cfg, glist, analysis=ana)
    close(torch.stack(ana["gates"]), z["eval_gates"])
    close(ana["time_gate_values"], z["eval_time_gate_values"])
    if z["eval_evolution"].size:
        ev = ana["evolution"]
        close([ev[k] for k in ("delta_mean", "delta_std", "dynamic_radius_mean", "static_radius_mean",
                               "base_radius_mean", "anchor_beta")], z["eval_evolution"])
    else:
        assert "evolution" not in ana
    sd64 = {k: (v.double().requires_grad_(k not in _BUFFERS and "running" not in k) if v.dtype == torch.float32
                else v) for k, v in sd.items()}
    le, lr, ls, lrad = om.hyperbolic_get_loss(sd64, cfg, glist, torch.from_numpy(z["batch"]), z["radius_target"])
    close([float(le), float(lr), 0.0, float(lrad)], z["loss_components"], 1e-5)
    tw = float(z["task_weight"])
    (tw * le + (1 - tw) * lr + ls.sum() + lrad).backward()
    norms = [float(v.grad.norm()) for v in sd64.values() if torch.is_tensor(v) and v.grad is not None]
    np.testing.assert_allclose(float(np.sqrt(np.sum(np.square(norms)))), float(z["grad_norm"]), rtol=1e-4)


@pytest.mark.parametrize("kind", ["union", "lorentz"])
def test_row_subgraph_restriction(kind):
    """oracle.graph.row_subgraph (the config-5 row pin of tests/test_gpu_config5_pin.py): the
    layer outputs of selected rows (hubs, ordinary rows, rows without in-edges) from the
    restricted graph, with the messages materialised in edge chunks, equal the whole-graph
    oracle's rows."""
    from regcn_amd.synthetic import zipf_triples
    rng = np.random.default_rng(3)
    V, R, d = 3000, 16, 8
    tr = zipf_triples(rng, V, R, 20000)
    g = og.build_sub_graph(V, R, tr)
    deg = g["in_deg"]
    order = np.argsort(-deg, kind="stable")
    rows = np.unique(np.concatenate([order[:3], rng.choice(np.flatnonzero(deg > 0), 50, replace=False),
                                     np.flatnonzero(deg == 0)[:5]]))
    assert (deg[rows] == 0).any()
    gen = torch.Generator().manual_seed(4)
    h = ops.exp0(0.3 * torch.randn(V, d, generator=gen, dtype=torch.float64), C)
    rel = 0.1 * torch.randn(2 * R, d, generator=gen, dtype=torch.float64)
    w = [torch.randn(d, d, generator=gen, dtype=torch.float64) / d ** 0.5 for _ in range(3)]
    gs, nodes = og.row_subgraph(V, R, tr, rows)
    np.testing.assert_array_equal(nodes[:rows.size], rows)
    if kind == "union":
        full = ol.union_layer(g, h, rel, *w, C, 0.15)
        part = ol.union_layer(gs, h[nodes], rel, *w, C, 0.15, edge_chunk=97)
    else:
        wb = torch.randn(2 * R, (d // 2) * 4, generator=gen, dtype=torch.float64) / 2
        full = ol.lorentz_layer(g, h, rel, wb, w[1], w[2], C, d // 2)
        part = ol.lorentz_layer(gs, h[nodes], rel, wb, w[1], w[2], C, d // 2, edge_chunk=97)
    np.testing.assert_allclose(part[:rows.size].numpy(), full[rows].numpy(), rtol=1e-10, atol=1e-12)
