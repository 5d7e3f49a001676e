"""HIP path vs the reference's golden vectors and the CPU oracle (-m gpu).

Tolerance: |delta| <= 1e-4 * max(1, |ref|) elementwise; indices exact."""
import numpy as np
import pytest
import torch

from gpu_helpers import C, MODEL_CASES, assert_close, build_hyperbolic_model

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("cname,c", [("c01", 0.01), ("c05", 0.05)])
def test_row_ops_vs_golden(golden, cname, c):
    from regcn_amd.hyperbolic_ops import HyperbolicOps as H, LorentzOps as L
    z = golden("ops.npz")
    x, v, y, rad = (t(z[cname + k]) for k in ("_x", "_v", "_y", "_rad"))
    assert_close(H.project_to_ball(x, c), z[cname + "_project"], what="project")
    assert_close(H.log_map_zero(x, c), z[cname + "_log0"], what="log0")
    assert_close(H.exp_map_zero(v, c), z[cname + "_exp0"], what="exp0")
    xb = H.project_to_ball(x, c)
    assert_close(H.mobius_add(xb, y, c), z[cname + "_mobius"], what="mobius")
    # atanh near the ball boundary amplifies fp32 rounding of |(-x)(+)y| by its relative
    # condition number k = z / ((1 - z^2) atanh z), z = sqrt(c)|.|; the tolerance scales by it.
    ref = np.asarray(z[cname + "_dist"], np.float64)
    zz = np.tanh(ref * np.sqrt(c) / 2)
    kappa = np.where(zz > 1e-6, zz / np.maximum((1 - zz ** 2) * np.arctanh(np.minimum(zz, 1 - 1e-12)), 1e-30), 1.0)
    got = H.hyperbolic_distance(xb, y, c).double().cpu().numpy()
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref)) / np.maximum(1.0, kappa)
    assert err.max() <= 1e-4, "dist condition-scaled error %.3g" % err.max()
    assert_close(H.get_radius(x), z[cname + "_radius"], what="radius")
    assert_close(H.apply_radius(y, rad, c), z[cname + "_apply_radius"], what="apply_radius")
    Lz = L.to_lorentz(y, c)
    assert_close(Lz, z[cname + "_to_lorentz"], what="to_lorentz")
    assert_close(L.to_poincare(Lz, c), z[cname + "_to_poincare"], what="to_poincare")


@pytest.mark.parametrize("d", [3, 64, 200, 256, 300])
def test_row_ops_any_width_vs_oracle(d):
    from oracle import ops as O
    from regcn_amd.hyperbolic_ops import HyperbolicOps as H
    g = torch.Generator().manual_seed(d)
    x = torch.randn(37, d, generator=g) * 0.3
    assert_close(H.log_map_zero(H.exp_map_zero(x.to(DEV), C), C), O.log0(O.exp0(x, C), C), what="roundtrip")
    assert_close(H.layer_norm_roundtrip(x.to(DEV), C), O.exp0(torch.nn.functional.normalize(O.log0(x, C)), C))


def _graph(z, prefix="", chunk=512, budget=None):
    """budget=1 sends every row with 2+ in-edges through the chunked pre-aggregation
    (and, with a small chunk, its fix-up pass) instead of the fused kernel's inline gather."""
    from regcn_amd import graph as G
    V, R = int(z[prefix + "meta"][0]), int(z[prefix + "meta"][1])
    g = G.build_sub_graph(V, R, z[prefix + "triples"], True, DEV, chunk_edges=chunk, tile_budget=budget)
    if budget == 1:
        assert g.n_heavy > 0
    return g


@pytest.mark.parametrize("gamma,gname", [(0.0, "g0"), (0.15, "g15")])
@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("chunk,budget", [(512, None), (3, 1), (512, 1)])
def test_union_layer_vs_golden(golden, gamma, gname, skip, chunk, budget):
    import torch.nn.functional as F
    from regcn_amd.hyperbolic_layers import HyperbolicUnionRGCNLayer
    z = golden("layer_union.npz")
    V, R, d = (int(v) for v in z["meta"])
    lay = HyperbolicUnionRGCNLayer(d, d, 2 * R, -1, c=C, activation=F.rrelu, self_loop=True, dropout=0.2,
                                   skip_connect=skip, radius_msg_gamma=gamma)
    lay.load_state_dict({k: torch.from_numpy(z["w_" + k]) for k in lay.state_dict()})
    lay = lay.to(DEV).eval()
    g = _graph(z, chunk=chunk, budget=budget)
    with torch.no_grad():
        y = lay(g, t(z["h"]), t(z["rel"]), prev_h=t(z["prev_h"]) if skip else None)
    assert_close(y, z["%s_%s_out" % (gname, "skip" if skip else "noskip")], what="union layer")


@pytest.mark.parametrize("chunk,budget", [(512, None), (2, 1)])
def test_euclid_layer_vs_golden(golden, chunk, budget):
    import torch.nn.functional as F
    from regcn_amd.layers import UnionRGCNLayer
    z = golden("layer_euclid.npz")
    V, R, d = (int(v) for v in z["meta"])
    lay = UnionRGCNLayer(d, d, 2 * R, -1, activation=F.rrelu, self_loop=True, dropout=0.2)
    lay.load_state_dict({k: torch.from_numpy(z["w_" + k]) for k in lay.state_dict()})
    lay = lay.to(DEV).eval()
    g = _graph(z, chunk=chunk, budget=budget)
    g.ndata["h"] = t(z["h"])
    with torch.no_grad():
        y = lay(g, [], t(z["rel"]))
    assert_close(y, z["out"], what="euclid layer")


@pytest.mark.parametrize("tag,skip", [("s2", False), ("s2", True), ("s4", False), ("s1", False), ("s20", False)])
@pytest.mark.parametrize("chunk,budget", [(512, None), (5, 1), (512, 3)])
def test_lorentz_layer_vs_golden(golden, tag, skip, chunk, budget):
    import torch.nn.functional as F
    from regcn_amd.hyperbolic_layers import LorentzRGCNLayer
    z = golden("layer_lorentz.npz")
    V, R, d, nb = (int(v) for v in z[tag + "_meta"])
    lay = LorentzRGCNLayer(d, d, 2 * R, nb, c=C, activation=F.rrelu, self_loop=True, dropout=0.2,
                           skip_connect=skip)
    sd = {k: torch.from_numpy(z[tag + "_w_" + k]) for k in lay.state_dict()}
    lay.load_state_dict(sd)
    lay = lay.to(DEV).eval()
    g = _graph(z, tag + "_", chunk=chunk, budget=budget)
    with torch.no_grad():
        y = lay(g, t(z[tag + "_h"]), t(z[tag + "_rel"]), prev_h=t(z[tag + "_prev_h"]) if skip else None)
    assert_close(y, z[tag + ("_skip" if skip else "_noskip") + "_out"], what="lorentz layer")


@pytest.mark.parametrize("tag", list(MODEL_CASES))
def test_hyperbolic_model_predict_vs_golden(golden, tag):
    z = golden("model_%s.npz" % tag)
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, DEV)
    with torch.no_grad():
        embs, _, h0, _, _ = m.forward(glist, None, True)
        all_tr, score, score_rel = m.predict(glist, R, None, torch.from_numpy(z["test"]).to(DEV), True)
    np.testing.assert_array_equal(all_tr.cpu().numpy(), z["all_triples"])
    if "embs" in z:
        assert_close(torch.stack(embs), z["embs"], what="history_embs")
    else:  # the dataset-shaped goldens keep the last history embedding
        assert_close(embs[-1], z["embs_last"], what="last history embedding")
    assert_close(h0, z["h0"], what="h_0")
    assert_close(score, z["score"], what="entity score")
    assert_close(score_rel, z["score_rel"], what="relation score")
    if "r512" in tag or "e80k" in tag:
        assert any(g.n_heavy > 0 for g in glist), "the golden must reach the pre-aggregated hub rows"


@pytest.mark.parametrize("V,R,T,hub", [(500, 10, 300, False), (4000, 40, 2000, True), (300, 60, 5, False)])
def test_relation_gru_two_phase(V, R, T, hub):
    """regcn_relation_gru_pre_f32 + regcn_relation_gru_x_f32 against torch.nn.GRUCell on
    [emb_rel | mean over the r_to_e span of x] (hyperbolic_model.py:797-818), fp32,
    tolerance 1e-4 * max(1, |ref|); absent relations (mean 0), spans over the in-kernel
    limit (precomputed means) and a single-triple relation covered; also the one-launch
    kernel (regcn_relation_gru_f32) on the same inputs."""
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import relation_gru_pre, relation_gru_step, relation_gru_x
    rng = np.random.default_rng(V)
    tri = np.stack([rng.integers(0, V, T), rng.integers(0, R // 2, T), rng.integers(0, V, T)], 1)
    if hub:
        tri[:300, 1] = 3  # a relation whose span is longer than the in-kernel limit
    g = G.build_sub_graph(V, R, tri, True, DEV)
    d = 200
    torch.manual_seed(V)
    gru = torch.nn.GRUCell(2 * d, d).to(DEV)
    x = torch.randn(V, d, device=DEV)
    emb = torch.randn(2 * R, d, device=DEV)
    h_prev = torch.randn(2 * R, d, device=DEV)
    with torch.no_grad():
        got = relation_gru_x(gru, x, g, h_prev, relation_gru_pre(gru, emb, h_prev))
        one = relation_gru_step(gru, emb, x, g, h_prev)
        means = torch.zeros(2 * R, d, device=DEV)
        r2e = g.r_to_e.to(DEV) if torch.is_tensor(g.r_to_e) else torch.tensor(g.r_to_e, device=DEV)
        for (a, b), r in zip(g.r_len, g.uniq_r):
            means[int(r)] = x[r2e[a:b]].mean(0)
        ref = gru(torch.cat([emb, means], 1), h_prev)
    assert_close(got, ref.cpu().numpy(), what="two-phase GRU")
    assert_close(one, ref.cpu().numpy(), what="one-launch GRU")


@pytest.mark.parametrize("encoder,layers,skip,self_loop,ln", [
    ("lgcn", 2, False, True, False), ("hyperbolic_uvrgcn", 2, False, True, True),
    ("lgcn", 2, True, True, False), ("lgcn", 2, True, False, True), ("hyperbolic_uvrgcn", 1, False, True, False),
])
def test_phase_pipeline_bitwise(encoder, layers, skip, self_loop, ln):
    """_forward_phases (three phase launches per timestep, csrc/timestep.hip; without the memo
    also with the rows without in-edges in their own side-stream launch, csrc/window.hip), with and
    without the memoised pristine states (rows without an in-edge so far: copied from
    F^t(initial state), csrc/window.hip over all rows), equals the per-layer launches bit for
    bit, history embeddings, tangent caches and h_0 included; the window holds an empty
    snapshot (no in-edge rows) and a one-triple one."""
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    from regcn_amd.synthetic import snapshot_series
    from regcn_amd.tangent import tangent_of
    V, R, d = 3000, 50, 200  # R2 = 100 = num_bases: d / num_bases = 2 (lgcn blocks)
    snaps = snapshot_series(3, V, R, 4, 300)
    snaps[1] = np.zeros((0, 3), np.int64)
    snaps[2] = snaps[2][:1]
    torch.manual_seed(0)
    m = HyperbolicRecurrentRGCN("roth", encoder, V, R, 0, 0, d, "sub", 4, num_bases=100, num_hidden_layers=layers,
                                dropout=0.2, c=C, self_loop=self_loop, skip_connect=skip, layer_norm=ln,
                                entity_prediction=True, relation_prediction=True, use_cuda=True,
                                radius_target=np.random.default_rng(0).uniform(0.5, 3, V).astype(np.float32),
                                radius_msg_gamma=0.15).to(DEV).eval()
    glist = [G.build_sub_graph(V, R, s, True, DEV) for s in snaps]
    res = {}
    for mode in ("memo", "split", "phases", "layers"):
        m.use_phases = mode != "layers"
        m.memo_pristine = mode == "memo"
        m.split_zero_rows = mode == "split"  # rows without in-edges in regcn_zero_step_f32
        with torch.no_grad():
            embs, _, h0, _, _ = m.forward(glist, None, True)
        torch.cuda.synchronize()
        res[mode] = [e.clone() for e in embs] + [tangent_of(e, C)[k].clone() for e in embs for k in (0, 1)] + [h0]
    m.memo_pristine = HyperbolicRecurrentRGCN.memo_pristine
    m.split_zero_rows = HyperbolicRecurrentRGCN.split_zero_rows
    for mode in ("memo", "split", "phases"):
        for a, b in zip(res[mode], res["layers"]):
            assert torch.equal(a, b), mode


@pytest.mark.parametrize("R,d,means_first", [(13, 200, False), (13, 72, True), (50, 200, True), (64, 100, False)])
def test_phase_gru_parts_on_eight_waves(R, d, means_first, monkeypatch):
    """The relation-GRU parts (csrc/gru_parts.h, written for 4 waves) hosted by the 8-wave phase
    workgroups (timestep.hip, -DREGCN_ROWTILE_WAVES=8): waves 4-7 run the same barrier
    sequence with their work predicated off.  R2 = 26 / 100 / 128 relation rows (a last GRU row
    tile of 10 / 4 / 16 rows), the relation means inline in the x-part (stage_rel_means, its
    own barrier) or precomputed (x_mean, the other staging path); phase launches equal the
    per-layer launches bit for bit, and two runs of the phases equal each other.  (Round 5's
    hang and "memo" mismatches were waves 4-7 leaving the GRU parts early, so the workgroup's
    barriers no longer paired up.)"""
    from regcn_amd import graph as G
    from regcn_amd import hyperbolic_model as HM
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    from regcn_amd.synthetic import snapshot_series
    monkeypatch.setattr(HM, "REL_INLINE_MAX_SPAN", -1 if means_first else 1 << 30)
    V, T = 2000, 3
    snaps = snapshot_series(11, V, R, T, 400)
    torch.manual_seed(2)
    m = HyperbolicRecurrentRGCN("roth", "hyperbolic_uvrgcn", V, R, 0, 0, d, "sub", T, num_bases=d // 2,
                                num_hidden_layers=2, dropout=0.2, c=C, self_loop=True, layer_norm=False,
                                entity_prediction=True, relation_prediction=True, use_cuda=True,
                                radius_msg_gamma=0.15).to(DEV).eval()
    m.param_caches = m.memo_pristine = False
    glist = [G.build_sub_graph(V, R, s, True, DEV) for s in snaps]
    assert all(HM._means_first(g) == means_first for g in glist)
    res = {}
    for mode in ("phases", "phases_again", "layers"):
        m.use_phases = mode != "layers"
        with torch.no_grad():
            embs, _, h0, _, _ = m.forward(glist, None, True)
        torch.cuda.synchronize()
        res[mode] = [e.clone() for e in embs] + [h0.clone()]
    for mode in ("phases", "phases_again"):
        for a, b in zip(res[mode], res["layers"]):
            assert torch.equal(a, b), mode


@pytest.mark.parametrize("encoder,ln", [("lgcn", False), ("hyperbolic_uvrgcn", True)])
def test_shared_parameter_states_bitwise(encoder, ln):
    """A batch of independent predicts inside HyperbolicRecurrentRGCN.shared_parameter_states
    (parameter-only states computed once: initial state, GRU pre-half, pristine rows copied
    from the batch's cold chain) returns exactly what each predict computes alone, every
    parameter cache off; two batches in a row (nothing carried over), windows sharing
    snapshots, an empty snapshot among them."""
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    from regcn_amd.synthetic import snapshot_series
    V, R, d, T = 2500, 50, 200, 3
    snaps = snapshot_series(5, V, R, 7, 250)
    snaps[3] = np.zeros((0, 3), np.int64)
    torch.manual_seed(1)
    m = HyperbolicRecurrentRGCN("roth", encoder, V, R, 0, 0, d, "sub", T, num_bases=100, num_hidden_layers=2,
                                dropout=0.2, c=C, self_loop=True, layer_norm=ln, entity_prediction=True,
                                relation_prediction=True, use_cuda=True,
                                radius_target=np.random.default_rng(1).uniform(0.5, 3, V).astype(np.float32),
                                radius_msg_gamma=0.15).to(DEV).eval()
    m.param_caches = m.memo_pristine = False
    glists = [[G.build_sub_graph(V, R, s, True, DEV) for s in snaps[i:i + T]] for i in range(4)]
    tests = [torch.from_numpy(snaps[i + T]).to(DEV) for i in range(4)]
    with torch.no_grad():
        alone = [[x.clone() for x in m.predict(gl, R, None, te, True)] for gl, te in zip(glists, tests)]
        for _ in range(2):
            with m.shared_parameter_states(T):
                batch = [[x.clone() for x in m.predict(gl, R, None, te, True)] for gl, te in zip(glists, tests)]
            torch.cuda.synchronize()
            for a, b in zip(alone, batch):
                for x, y in zip(a, b):
                    assert torch.equal(x, y)
    m.param_caches = HyperbolicRecurrentRGCN.param_caches
    m.memo_pristine = HyperbolicRecurrentRGCN.memo_pristine


@pytest.mark.parametrize("n_test,d", [(37, 200), (1, 200), (64, 256), (5, 12)])
def test_fused_roth_decoders(n_test, d):
    """HyperbolicRecurrentRGCN.predict with the two-launch RotH/RotHRel front
    (regcn_roth_queries_f32 on 4-query tiles + regcn_hyp_score_jobs_f32) against the
    per-decoder path (16-row query kernels on two streams + torch.cat): all_triples exact,
    scores within 1e-4 * max(1, |ref|) (the MFMA shapes differ, so do the summation orders),
    ranks of the targets equal; decoder weights drawn well away from their 1e-3 init so the
    reshape MLP and the projections matter.  B = 2 n_test is not a multiple of 4 in two cases."""
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    from regcn_amd.synthetic import snapshot_series
    V, R = 2000, 30
    snaps = snapshot_series(4, V, R, 7, 400)
    torch.manual_seed(n_test)
    m = HyperbolicRecurrentRGCN("roth", "hyperbolic_uvrgcn", V, R, 0, 0, d, "sub", 3, num_bases=10, num_hidden_layers=2,
                                dropout=0.2, c=C, self_loop=True, entity_prediction=True, relation_prediction=True,
                                use_cuda=True, radius_target=np.random.default_rng(0).uniform(0.5, 3, V).astype(np.float32),
                                radius_msg_gamma=0.15).to(DEV).eval()
    with torch.no_grad():
        for dec in (m.decoder_ob, m.rdecoder):
            for name, p in dec.named_parameters():
                if name.endswith("weight") or name.endswith("bias"):
                    p.normal_(0.0, 0.08)
        m.rdecoder.score_margin.fill_(0.7)
    glist = [G.build_sub_graph(V, R, s, True, DEV) for s in snaps[:3]]
    test = torch.from_numpy(snaps[3][:n_test]).to(DEV)
    res = {}
    for fused in (True, False):
        m.fused_decoders = fused
        with torch.no_grad():
            res[fused] = [x.clone() for x in m.predict(glist, R, None, test, True)]
        torch.cuda.synchronize()
    m.fused_decoders = HyperbolicRecurrentRGCN.fused_decoders
    assert torch.equal(res[True][0], res[False][0])
    assert_close(res[True][1], res[False][1].cpu().numpy(), what="entity score")
    assert_close(res[True][2], res[False][2].cpu().numpy(), what="relation score")
    at = res[False][0]
    for k, col in ((1, 2), (2, 1)):
        a, b = res[True][k], res[False][k]
        ra = (a > a.gather(1, at[:, col:col + 1])).sum(1)
        rb = (b > b.gather(1, at[:, col:col + 1])).sum(1)
        diff = (ra - rb).abs()
        assert int(diff.max()) <= 1 and int((diff > 0).sum()) <= 2  # near-ties may flip


@pytest.mark.parametrize("tag", ["uvrgcn_roth", "lgcn_roth", "uvrgcn_murp_nores", "uvrgcn_atth_beta",
                                 "lgcn_roth_bias_crel"])
def test_get_loss_vs_golden(golden, tag):
    z = golden("model_%s.npz" % tag)
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, DEV)
    with torch.no_grad():
        losses = m.get_loss(glist, torch.from_numpy(z["test"]).to(DEV), None, True)
    got = np.array([float(x) for x in losses])
    assert_close(got, z["losses"], what="losses")


@pytest.mark.parametrize("tag", ["noln", "ln", "ln_d200"])
def test_euclid_model_vs_golden(golden, tag):
    """RecurrentRGCN + ConvTransE (src/rrgcn.py:142-194); ln_d200: d = 200 at ICEWS14s' R = 230."""
    from regcn_amd import graph as G
    from regcn_amd.rrgcn import RecurrentRGCN
    z = golden("rrgcn_%s.npz" % tag)
    V, R, d, T = (int(v) for v in z["meta"])
    m = RecurrentRGCN("convtranse", "uvrgcn", V, R, 0, 0, d, "sub", T, num_bases=100, num_basis=100,
                      num_hidden_layers=2, dropout=0.2, self_loop=True, layer_norm=tag.startswith("ln"),
                      input_dropout=0.2, hidden_dropout=0.2, feat_dropout=0.2, entity_prediction=True,
                      relation_prediction=True, use_cuda=True, gpu=0)
    m.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd_")})
    m = m.to(DEV).eval()
    glist = [G.build_sub_graph(V, R, z["snap%d" % i], True, DEV) for i in range(T)]
    with torch.no_grad():
        embs, _, h0, _, _ = m.forward(glist, None, True)
        _, score, score_rel = m.predict(glist, R, None, torch.from_numpy(z["test"]).to(DEV), True)
    assert_close(torch.stack(embs), z["embs"], what="embs")
    assert_close(h0, z["h0"], what="h0")
    assert_close(score, z["score"], what="score")
    assert_close(score_rel, z["score_rel"], what="score_rel")


def test_score_and_ce_vs_golden(golden):
    from regcn_amd.hyperbolic_decoder import _chunked_hyperbolic_ce_loss as ce
    from regcn_amd.hyperbolic_decoder import _chunked_hyperbolic_dist_score as sc
    z = golden("score.npz")
    q, e, bias, scale, margin, cr, tgt = (t(z[k]) for k in ("q", "e", "bias", "scale", "margin", "c_r", "target"))
    assert_close(sc(q, e, None, C, 128, 256), z["score_plain"], what="plain")
    assert_close(sc(q, e, bias, C, 128, 256, score_scale=scale, score_margin=margin), z["score_bias"], what="bias")
    assert_close(sc(q, e, bias, C, 128, 256, score_scale=scale, score_margin=margin, query_curvature=cr,
                    use_hyperbolic_distance=True), z["score_crel"], what="crel")
    assert_close(sc(q, e, None, C, 128, 256, score_scale=scale, score_margin=margin, use_hyperbolic_distance=True),
                 z["score_dist"], what="dist")
    assert_close(ce(q, e, tgt, C, 256, candidate_bias=bias, score_scale=scale, score_margin=margin).reshape(1),
                 z["ce_bias"].reshape(1), what="ce")
    assert_close(ce(q, e, tgt, C, 256, candidate_bias=bias, score_scale=scale, score_margin=margin,
                    query_curvature=cr, use_hyperbolic_distance=True).reshape(1), z["ce_crel"].reshape(1),
                 what="ce crel")


# N % 4 == 0 stages the candidates permuted (a lane's four consecutive, one vector store per
# query row); other N keep the plain order (score.hip score_f32_body `perm`): both, with
# partial query and candidate tiles
@pytest.mark.parametrize("B,N,d", [(1, 1, 4), (5, 7, 12), (130, 1000, 200), (64, 64, 256), (160, 2048, 200),
                                   (300, 4099, 200), (129, 4160, 196)])
def test_score_shapes_vs_oracle(B, N, d):
    from oracle import model as OM
    from oracle import ops as O
    from regcn_amd.hyperbolic_decoder import _chunked_hyperbolic_dist_score as sc
    g = torch.Generator().manual_seed(B * 1000 + N)
    q = O.exp0(torch.randn(B, d, generator=g), C)
    e = O.exp0(torch.randn(N, d, generator=g), C)
    assert_close(sc(q.to(DEV), e.to(DEV), None, C, 128, 256), OM.dist_score(q, e, None, C), what="score")


@pytest.mark.parametrize("B,N,d,ranges", [(1, 1, 4, [(0, 1)]), (5, 700, 12, [(0, 300), (300, 301), (500, 700)]),
                                           (130, 3000, 200, [(0, 1000), (1000, 3000)]), (1024, 20000, 256, [(0, 20000)]),
                                           (256, 5000, 200, [(k * 500, k * 500 + 40 * k + 1) for k in range(10)])])
def test_fused_rank_count_matches_score_matrix(B, N, d, ranges):
    """regcn_hyp_rank_fused_f32 (score + count-greater in one launch, no score matrix) against
    regcn_hyp_score_f32 + the count over the score matrix: equal counts for thresholds at
    existing scores (ties at the threshold are not counted: strictly greater) and in between,
    over several candidate ranges (one launch for up to 8, accumulated past that:
    CandidateShard.fused_counts), with a per-
    candidate bias and the raw score scale; filter_hits: the listed answers above the threshold."""
    from regcn_amd.hyperbolic_decoder import _chunked_hyperbolic_dist_score as sc
    from regcn_amd.parallel import CandidateShard
    from oracle import ops as O
    g = torch.Generator().manual_seed(B + N + d)
    q = O.exp0(torch.randn(B, d, generator=g), C).to(DEV)
    e = O.exp0(torch.randn(N, d, generator=g), C).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    scale_raw = torch.tensor(0.7, device=DEV)
    margin = torch.tensor(1.3, device=DEV)
    S = sc(q, e, bias, C, 0, 0, score_scale=scale_raw, score_margin=margin, _raw_scale=True)
    pick = torch.randint(0, N, (B,), generator=g).to(DEV)
    thr = S.gather(1, pick[:, None]).flatten()
    thr[::3] = thr[::3] + 1e-3  # thresholds between scores too
    sh = CandidateShard(N, 0, 1, None, ranges=ranges)
    kw = dict(scale=scale_raw, margin=margin, raw_scale=True)
    got = sh.fused_counts(q, e, bias, C, thr, **kw)
    mask = torch.zeros(N, dtype=torch.bool, device=DEV)
    for a, b in ranges:
        mask[a:b] = True
    want = ((S > thr[:, None]) & mask[None, :]).sum(1).to(torch.int32)
    assert torch.equal(got, want)
    # filtered: 3 listed answers per query
    fl = torch.randint(0, N, (B, 3), generator=g)
    fp = np.arange(0, 3 * B + 1, 3)
    hits = sh.filter_hits(q, e, bias, C, thr, fp, fl.flatten().numpy(), **kw)
    fl = fl.to(DEV)
    want_h = ((S.gather(1, fl) > thr[:, None]) & mask[fl]).sum(1).to(torch.int32)
    assert torch.equal(hits, want_h)


def _zipf_snapshot(V, R, T, seed):
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, V + 1) ** 1.1
    p /= p.sum()
    perm = rng.permutation(V)
    return np.stack([perm[rng.choice(V, T, p=p)], rng.integers(0, R, T), perm[rng.choice(V, T, p=p)]], 1)


@pytest.mark.parametrize("chunk", [2, 64, 4096])
@pytest.mark.parametrize("euclid", [False, True])
def test_union_source_runs_match_edge_sums(euclid, chunk):
    """regcn_union_aggregate_src_runs_f32 (a hub row's duplicate sources gathered once:
    count * w * x[src]) against regcn_union_aggregate_f32 over the CSR edge order on the same
    hub chunks.  The snapshot repeats triples (one source 300 times into a hub under many
    relations), so source runs cross 64-edge batches and chunk ends.  Also pins the
    row/source order: each row's CSR span sorted by source."""
    from regcn_amd import _lib
    from regcn_amd import graph as G
    V, R, d, gamma = 3000, 60, 200, 0.15
    rng = np.random.default_rng(11)
    tr = _zipf_snapshot(V, R, 20000, 5)
    hub = int(np.bincount(tr[:, 2], minlength=V).argmax())
    rep = np.stack([np.full(300, 17), rng.integers(0, R, 300), np.full(300, hub)], 1)
    tr = np.concatenate([tr, rep, tr[:2000]])
    g = G.build_sub_graph(V, R, tr, True, DEV, chunk_edges=chunk, tile_budget=64)
    assert g.n_heavy > 0
    wk = g.work()
    rowptr = wk["rowptr"].cpu().numpy()
    cs = wk["col_src"].cpu().numpy()
    csr_dst = np.repeat(np.arange(V), np.diff(rowptr))
    ss = g.row_src_cols()
    np.testing.assert_array_equal(ss.cpu().numpy(), cs[np.lexsort((cs, csr_dst))])
    gen = torch.Generator().manual_seed(2)
    x = (torch.randn(V, d, generator=gen) * 0.3).to(DEV)
    r = x.norm(dim=1).contiguous()
    rel = (torch.randn(2 * R, d, generator=gen) * 0.1).to(DEV)
    hc, hf = wk["heavy_chunks"], wk["heavy_fixups"]
    part = torch.empty(max(g.heavy_slots, 1), d + 4, device=DEV)
    f, i = _lib.fptr, _lib.iptr
    ref = torch.zeros(V, d, device=DEV)
    got = torch.zeros(V, d, device=DEV)
    if euclid:
        _lib.call("regcn_euclid_aggregate_f32", f(x), f(rel), i(wk["col_src"]), i(wk["col_type"]), f(wk["norm"]),
                  i(hc), hc.shape[0], i(hf), hf.shape[0], d, f(part), d + 4, f(ref), _lib.stream())
    else:
        _lib.call("regcn_union_aggregate_f32", f(x), f(r), f(rel), i(wk["col_src"]), i(wk["col_type"]),
                  f(wk["norm"]), i(hc), hc.shape[0], i(hf), hf.shape[0], gamma, d, f(part), d + 4, f(ref),
                  _lib.stream())
    ct_s, ct_t = g.row_type_cols()
    _lib.call("regcn_union_aggregate_src_runs_f32", f(x), None if euclid else f(r), f(rel), i(ct_s), i(ct_t), i(ss),
              f(wk["norm"]), i(hc), hc.shape[0], i(hf), hf.shape[0], gamma, int(euclid), d, f(part), d + 4, f(got),
              _lib.stream())
    torch.cuda.synchronize()
    heavy = torch.from_numpy(np.unique(hc.cpu().numpy()[:, 0])).long().to(DEV)
    assert got[heavy].abs().max() > 0
    assert_close(got, ref, what="source-run union aggregation")


@pytest.mark.parametrize("kind", ["union", "euclid"])
def test_layer_item_source_runs(kind):
    """The fused layer with its inline items in (row, source) order (regcn_layer_desc.
    item_src_runs: a row's duplicate sources gathered once, count * w * x[src]) against the
    oracle and against the CSR-order items; the snapshot repeats triples so light rows have
    source runs, and crosses the hub budget.  Also pins the item order: each row's items
    sorted by source, tiles unchanged."""
    import torch.nn.functional as F
    from oracle import graph as OG
    from oracle import layers as OL
    from oracle import ops as O
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_layers import HyperbolicUnionRGCNLayer
    from regcn_amd.layers import UnionRGCNLayer
    V, R, d = 3000, 60, 200
    tr = _zipf_snapshot(V, R, 20000, 9)
    tr = np.concatenate([tr, tr[:6000], tr[:1500, ::-1]])  # repeated triples and swapped pairs
    tr[-1500:, 1] = tr[-1500:, 1] % R
    g = G.build_sub_graph(V, R, tr, True, DEV)
    assert g.n_heavy > 0
    wk = g.work()
    isrc, itl = g.item_src_cols()
    tiles = wk["tiles"].cpu().numpy()
    iptr = wk["item_ptr"].cpu().numpy()
    rowpos = np.repeat(tiles[:, 0], np.diff(iptr)) + (wk["item_tl"].cpu().numpy() & 15)
    order = np.lexsort((wk["item_src"].cpu().numpy(), rowpos))
    np.testing.assert_array_equal(isrc.cpu().numpy(), wk["item_src"].cpu().numpy()[order])
    np.testing.assert_array_equal(itl.cpu().numpy(), wk["item_tl"].cpu().numpy()[order])
    s = isrc.cpu().numpy()
    assert (s[1:] == s[:-1]).sum() > 1000  # source runs inside rows
    og = OG.build_sub_graph(V, R, tr)
    gen = torch.Generator().manual_seed(4)
    rel = torch.randn(2 * R, d, generator=gen) * 0.1
    torch.manual_seed(0)
    if kind == "union":
        h = O.exp0(torch.randn(V, d, generator=gen) * 0.5, C)
        lay = HyperbolicUnionRGCNLayer(d, d, 2 * R, -1, c=C, activation=F.rrelu, self_loop=True,
                                       radius_msg_gamma=0.15).eval()
        ref = OL.union_layer(og, h, rel, lay.weight_neighbor.detach(), lay.loop_weight.detach(),
                             lay.evolve_loop_weight.detach(), C, 0.15)
        run = lambda: lay.to(DEV)(g, h.to(DEV), rel.to(DEV))  # noqa: E731
    else:
        lay = UnionRGCNLayer(d, d, 2 * R, -1, activation=F.rrelu, self_loop=True).eval()
        hx = torch.randn(V, d, generator=gen) * 0.1
        ref = OL.euclid_union_layer(og, hx, rel, lay.weight_neighbor.detach(), lay.loop_weight.detach(),
                                    lay.evolve_loop_weight.detach())
        def run():
            g.ndata["h"] = hx.to(DEV)  # the layer replaces it with its output
            return lay.to(DEV)(g, [], rel.to(DEV))
    outs = {}
    for on in (True, False):
        g.item_src_runs = on
        with torch.no_grad():
            outs[on] = run().clone()
    g.item_src_runs = None
    assert_close(outs[True], ref, what=kind + " layer, item source runs")
    assert_close(outs[True], outs[False], what=kind + " layer, item source runs vs CSR items")


@pytest.mark.parametrize("chunk", [None, 2])
@pytest.mark.parametrize("kind", ["union", "lorentz", "euclid"])
def test_layers_with_hubs_vs_oracle(kind, chunk):
    """Zipf snapshot with hubs over the tile budget (pre-aggregated + fixups) next to
    inline-gathered rows, at d = 200 / num_bases = 100 (the bench shape).  chunk = 2 gives
    the hubs hundreds of partial slots: their fix-ups go through the first-level groups."""
    import torch.nn.functional as F
    from oracle import graph as OG
    from oracle import layers as OL
    from oracle import ops as O
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_layers import HyperbolicUnionRGCNLayer, LorentzRGCNLayer
    from regcn_amd.layers import UnionRGCNLayer
    V, R, T, d = 3000, 60, 20000, 200  # 2R >= num_bases = 100 (else the reference clamps num_bases)
    tr = _zipf_snapshot(V, R, T, 7)
    g = G.build_sub_graph(V, R, tr, True, DEV, chunk_edges=chunk)
    assert g.n_heavy > 0 and g.heavy_slots > 0
    if chunk == 2:
        assert (g._host["heavy_fixups"][:, 3] > 0).any()
    og = OG.build_sub_graph(V, R, tr)
    gen = torch.Generator().manual_seed(3)
    h = O.exp0(torch.randn(V, d, generator=gen) * 0.5, C)
    rel = torch.randn(2 * R, d, generator=gen) * 0.1
    torch.manual_seed(0)
    if kind == "union":
        lay = HyperbolicUnionRGCNLayer(d, d, 2 * R, -1, c=C, activation=F.rrelu, self_loop=True, dropout=0.2,
                                       radius_msg_gamma=0.15).eval()
        ref = OL.union_layer(og, h, rel, lay.weight_neighbor.detach(), lay.loop_weight.detach(),
                             lay.evolve_loop_weight.detach(), C, 0.15)
        with torch.no_grad():
            y = lay.to(DEV)(g, h.to(DEV), rel.to(DEV))
    elif kind == "lorentz":
        lay = LorentzRGCNLayer(d, d, 2 * R, 100, c=C, activation=F.rrelu, self_loop=True, dropout=0.2).eval()
        ref = OL.lorentz_layer(og, h, rel, lay.weight.detach(), lay.loop_weight.detach(),
                               lay.evolve_loop_weight.detach(), C, 100)
        with torch.no_grad():
            y = lay.to(DEV)(g, h.to(DEV), rel.to(DEV))
    else:
        lay = UnionRGCNLayer(d, d, 2 * R, -1, activation=F.rrelu, self_loop=True, dropout=0.2).eval()
        hx = torch.randn(V, d, generator=gen) * 0.1
        ref = OL.euclid_union_layer(og, hx, rel, lay.weight_neighbor.detach(), lay.loop_weight.detach(),
                                    lay.evolve_loop_weight.detach())
        g.ndata["h"] = hx.to(DEV)
        with torch.no_grad():
            y = lay.to(DEV)(g, [], rel.to(DEV))
    assert_close(y, ref, what=kind + " layer with hubs")


@pytest.mark.parametrize("tag", ["lgcn_roth_bias_crel", "uvrgcn_roth", "lgcn_roth"])
def test_predict_is_deterministic(golden, tag):
    """Bitwise-identical reruns (no atomics, no uninitialised reads): the fused kernels
    combine partial sums in a fixed order."""
    z = golden("model_%s.npz" % tag)
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, DEV)
    test = torch.from_numpy(z["test"]).to(DEV)
    with torch.no_grad():
        runs = [m.predict(glist, R, None, test, True) for _ in range(3)]
    for _, s, sr in runs:
        assert torch.isfinite(s).all() and torch.isfinite(sr).all()
        assert torch.equal(s, runs[0][1]) and torch.equal(sr, runs[0][2])


@pytest.mark.parametrize("tag", ["uvrgcn_roth", "lgcn_roth"])
def test_roth_query_kernel_matches_torch_sequence(golden, tag):
    """regcn_roth_query_f32 / regcn_roth_rel_query_f32 against the same decoders run op by
    op on torch (hyperbolic_decoder.py:1065-1085, :1223-1243)."""
    from regcn_amd.hyperbolic_decoder import _RelDecoderBase
    z = golden("model_%s.npz" % tag)
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, DEV)
    test = torch.from_numpy(z["test"]).to(DEV)
    with torch.no_grad():
        emb_l, _, r_emb, _, _ = m.forward(glist, None, True)
        emb = emb_l[-1]
        inv = test.flip(1)
        inv[:, 1] += R
        at = torch.cat([test, inv])
        dec, rdec = m.decoder_ob, m.rdecoder
        q = dec._query(emb, r_emb, at)
        s_rel = rdec.forward(emb, r_emb, at)
        dec._torch_query = True
        q_t = dec._query(emb, r_emb, at)
        dec._torch_query = False
        s_rel_t = _RelDecoderBase.forward(rdec, emb, r_emb, at)
    assert_close(q, q_t, what="RotH query")
    assert_close(s_rel, s_rel_t, what="RotHRel scores")


@pytest.mark.parametrize("kind", ["lorentz", "union", "euclid"])
@pytest.mark.parametrize("partition,world", [("edge", 2), ("edge", 3), ("owner", 2), ("owner", 3)])
def test_sharded_layer_ranks_simulated(kind, partition, world):
    """Both multi-GPU partitions with the ranks run one after another on this device and
    the collectives done by hand (sum of partials / union of node blocks): equal to the
    unpartitioned layer (parallel.py)."""
    import torch.nn.functional as F
    from oracle import ops as O
    from regcn_amd import _lib
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_layers import HyperbolicUnionRGCNLayer, LorentzRGCNLayer, run_layer
    from regcn_amd.layers import UnionRGCNLayer
    from regcn_amd.parallel import ShardedGraph
    from regcn_amd.tangent import tangent_of
    from regcn_amd.weights import packed
    V, R, d = 3000, 60, 200
    g = G.build_sub_graph(V, R, _zipf_snapshot(V, R, 20000, 11), True, DEV)
    gen = torch.Generator().manual_seed(4)
    rel = (torch.randn(2 * R, d, generator=gen) * 0.1).to(DEV)
    torch.manual_seed(1)
    if kind == "lorentz":
        lay = LorentzRGCNLayer(d, d, 2 * R, 100, c=C, activation=F.rrelu, self_loop=True).to(DEV).eval()
        mode, wn, wrel, nb, gamma = _lib.AGG_LORENTZ, None, lay.weight.detach().contiguous(), 100, 0.0
    elif kind == "union":
        lay = HyperbolicUnionRGCNLayer(d, d, 2 * R, c=C, activation=F.rrelu, self_loop=True,
                                       radius_msg_gamma=0.15).to(DEV).eval()
        mode, wn, wrel, nb, gamma = _lib.AGG_UNION, lay.weight_neighbor, None, 0, 0.15
    else:
        lay = UnionRGCNLayer(d, d, 2 * R, -1, activation=F.rrelu, self_loop=True).to(DEV).eval()
        mode, wn, wrel, nb, gamma = _lib.AGG_EUCLID, lay.weight_neighbor, None, 0, 0.0
    euclid = kind == "euclid"
    if euclid:
        x = (torch.randn(V, d, generator=gen) * 0.1).to(DEV)
        r = None
    else:
        h = O.exp0(torch.randn(V, d, generator=gen) * 0.5, C).to(DEV)
        x, r = tangent_of(h, C)
    args = (rel, wrel, nb, gamma, wn, lay.loop_weight, lay.evolve_loop_weight, None, None, None, None, C)
    with torch.no_grad():
        ref = run_layer(mode, g, x, r, *args, euclid=euclid)[0]
        shards = [ShardedGraph(g, partition, rank=k, world=world) for k in range(world)]
        if partition == "edge":
            Psum = sum(s.edge_partials(mode, x, r, rel, wrel, nb, gamma, C) for s in shards)
            agg = shards[0].edge_finish(mode, Psum, x, r, rel, wrel, nb, gamma, C)
            got = run_layer(_lib.AGG_NONE, g, x, r, *args, euclid=euclid, agg=agg)[0]
        else:
            got = torch.full_like(x, float("nan"))
            xn, rn = torch.empty_like(x), torch.empty(V, device=DEV)
            for s in shards:
                for _, view in s.views:  # the rank's pipeline chunks of owned rows
                    run_layer(mode, view, x, r, *args, euclid=euclid, out=(got, xn, rn))
    assert torch.isfinite(got).all()
    assert_close(got, ref, what="%s %s x%d" % (kind, partition, world))


@pytest.mark.parametrize("partition", ["edge", "owner"])
def test_sharded_graph_model_predict_world1(golden, partition):
    """HyperbolicRecurrentRGCN.predict over ShardedGraph snapshots (the dispatch the
    torchrun job uses; world 1 without a process group) matches the golden."""
    from regcn_amd.parallel import ShardedGraph
    tag = "lgcn_roth"
    z = golden("model_%s.npz" % tag)
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, DEV)
    sg = [ShardedGraph(g, partition) for g in glist]
    with torch.no_grad():
        _, score, score_rel = m.predict(sg, R, None, torch.from_numpy(z["test"]).to(DEV), True)
    assert_close(score, z["score"], what="entity score")
    assert_close(score_rel, z["score_rel"], what="relation score")


def test_total_rank_vs_golden(golden):
    """get_total_rank (raw + time-filtered, entity and relation) against the reference's
    ranks and MRRs (rgcn/utils.py:136-166) on the golden scores."""
    from regcn_amd.ranking import get_total_rank, load_all_answers_for_filter
    z = golden("rank.npz")
    V, R = (int(v) for v in z["meta"])
    tr = torch.from_numpy(z["all_triples"]).to(DEV)
    ans_e = load_all_answers_for_filter(z["snap"], R, False)
    ans_r = load_all_answers_for_filter(z["snap"], R, True)
    mf, m, rank, frank = get_total_rank(tr, t(z["score"]), ans_e, 1000)
    np.testing.assert_array_equal(rank.cpu().numpy(), z["rank"])
    np.testing.assert_array_equal(frank.cpu().numpy(), z["frank"])
    mfr, mr, rank_r, frank_r = get_total_rank(tr, t(z["score_rel"]), ans_r, 1000, rel_predict=1)
    np.testing.assert_array_equal(rank_r.cpu().numpy(), z["rank_r"])
    np.testing.assert_array_equal(frank_r.cpu().numpy(), z["frank_r"])
    np.testing.assert_allclose([m, mf, mr, mfr], z["mrr"], rtol=1e-6)


def test_multistep_history_from_filtered_scores(golden):
    """--multi-step (hyperbolic_main.py:135-149): get_total_rank leaves the other true
    answers at -1e7 in the score (rgcn/utils.py:51-75) and construct_snap(_r) takes the
    next history snapshot's top-k from those filtered scores; both against the reference."""
    from regcn_amd.ranking import construct_snap, construct_snap_r, get_total_rank, load_all_answers_for_filter
    z, zm = golden("rank.npz"), golden("multistep.npz")
    V, R = (int(v) for v in z["meta"])
    k = int(zm["topk"][0])
    tr = torch.from_numpy(z["all_triples"]).to(DEV)
    score, score_rel = t(z["score"]).clone(), t(z["score_rel"]).clone()
    get_total_rank(tr, score, load_all_answers_for_filter(z["snap"], R, False), 1000)
    get_total_rank(tr, score_rel, load_all_answers_for_filter(z["snap"], R, True), 1000, rel_predict=1)
    np.testing.assert_array_equal(score.cpu().numpy(), zm["filtered_score"])
    np.testing.assert_array_equal(score_rel.cpu().numpy(), zm["filtered_score_rel"])
    np.testing.assert_array_equal(construct_snap(tr, V, R, score, k), zm["snap_e"])
    np.testing.assert_array_equal(construct_snap_r(tr, V, R, score_rel, k), zm["snap_r"])


@pytest.mark.parametrize("world", [1, 3, 8])
def test_candidate_sharded_decoder(world):
    """SURVEY.md §8(e) decoder: each rank scores a slice of the candidates; the ranks (raw and
    filtered) summed over the slices equal the unsharded ranks exactly, the cross entropy
    matches the unsharded fused CE.  The ranks are simulated on one GPU (group=None) and
    combined here with the same reductions the collectives apply."""
    from regcn_amd import ranking
    from regcn_amd.hyperbolic_decoder import _chunked_hyperbolic_ce_loss, _chunked_hyperbolic_dist_score
    from regcn_amd.parallel import CandidateShard
    g = torch.Generator().manual_seed(world)
    B, N, d = 300, 5003, 200
    q = (torch.randn(B, d, generator=g) * 0.3).to(DEV)
    e = (torch.randn(N, d, generator=g) * 0.3).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    tgt = torch.randint(0, N, (B,), generator=g).to(DEV)
    scale, margin = torch.tensor(1.3, device=DEV), torch.tensor(0.7, device=DEV)
    # filter lists: a few random other answers per query
    rng = np.random.default_rng(world)
    ptr, idx = [0], []
    for b in range(B):
        o = rng.integers(0, N, size=rng.integers(0, 6))
        idx.extend(sorted(set(o.tolist()) - {int(tgt[b])}))
        ptr.append(len(idx))
    fp, fi = np.asarray(ptr, np.int32), np.asarray(idx, np.int32)
    full = _chunked_hyperbolic_dist_score(q, e, bias, C, 0, 0, score_scale=scale, score_margin=margin)
    want_raw, want_flt = ranking.ranks(full, tgt, fp, fi)
    raw = torch.zeros(B, dtype=torch.long, device=DEV)
    flt = torch.zeros(B, dtype=torch.long, device=DEV)
    lses = []
    for rank in range(world):
        sh = CandidateShard(N, rank, world)
        ts = sh.target_scores(q, e, bias, tgt, C, scale, margin)
        assert torch.equal(ts, full[torch.arange(B, device=DEV), tgt])  # the same bits
        r, f = sh.ranks(sh.scores(q, e, bias, C, scale, margin), ts, fp, fi)
        raw += r - 1
        flt += f - 1
        lses.append(sh.local_lse(q, e, bias, C, scale, margin))
    assert torch.equal(raw + 1, want_raw) and torch.equal(flt + 1, want_flt)
    lse = torch.logsumexp(torch.stack(lses), 0)
    loss = (lse - full[torch.arange(B, device=DEV), tgt]).mean()
    ref = _chunked_hyperbolic_ce_loss(q, e, tgt, C, 0, candidate_bias=bias, score_scale=scale, score_margin=margin)
    assert abs(float(loss) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))


@pytest.mark.parametrize("N", [1, 3, 7, 1023, 4099, 130001])
def test_rank_counts_vs_torch(N):
    """regcn_rank_f32 (k_rank: one workgroup per query, 16-B body loads between a scalar head
    and tail -- a row starts anywhere when N % 4 != 0) against torch's count of the scores above
    the target's, raw and filtered; quantised scores, so ties with the target occur."""
    from regcn_amd import ranking
    g = torch.Generator().manual_seed(N)
    B = 37
    S = (torch.randint(0, 64, (B, N), generator=g).float() / 8.0).to(DEV)
    tgt = torch.randint(0, N, (B,), generator=g)
    rng = np.random.default_rng(N)
    ptr, idx = [0], []
    for b in range(B):
        o = rng.integers(0, N, size=rng.integers(0, 9))
        idx.extend(sorted(set(o.tolist()) - {int(tgt[b])}))
        ptr.append(len(idx))
    fp, fi = np.asarray(ptr, np.int32), np.asarray(idx, np.int32)
    raw, flt = ranking.ranks(S, tgt, fp, fi)
    Sc = S.cpu()
    ts = Sc[torch.arange(B), tgt].unsqueeze(1)
    want = 1 + (Sc > ts).sum(1)
    wf = want.clone()
    for b in range(B):
        cols = torch.from_numpy(fi[fp[b]:fp[b + 1]].astype(np.int64))
        wf[b] -= int((Sc[b, cols] > ts[b]).sum())
    assert torch.equal(raw.cpu(), want) and torch.equal(flt.cpu(), wf)


@pytest.mark.parametrize("d", [8, 200, 252])
def test_pack_unpack_rows(d):
    """regcn_pack_rows_f32 / regcn_unpack_rows_f32 (the owner partition's exchange records):
    records [x row, |h|, 0, 0, 0] of the listed rows, bit for bit, and the unpack writes exactly
    the listed rows back."""
    from regcn_amd.parallel import pack_rows, unpack_rows
    g = torch.Generator().manual_seed(d)
    V = 5000
    x = torch.randn(V, d, generator=g).to(DEV)
    r = torch.rand(V, generator=g).to(DEV)
    ids = torch.randperm(V, generator=g)[:1237].to(DEV)
    buf = pack_rows(x, r, ids)
    assert buf.shape == (1237, d + 4)
    assert torch.equal(buf[:, :d], x[ids]) and torch.equal(buf[:, d], r[ids])
    assert torch.equal(buf[:, d + 1:], torch.zeros(1237, 3, device=DEV))
    x2 = torch.full_like(x, float("nan"))
    r2 = torch.full_like(r, float("nan"))
    unpack_rows(buf, ids, x2, r2)
    hit = torch.zeros(V, dtype=torch.bool, device=DEV)
    hit[ids] = True
    assert torch.equal(x2[hit], x[hit]) and torch.equal(r2[hit], r[hit])
    assert torch.isnan(x2[~hit]).all() and torch.isnan(r2[~hit]).all()
    empty = torch.zeros(0, dtype=torch.int64, device=DEV)
    assert pack_rows(x, r, empty).shape == (0, d + 4)


@pytest.mark.parametrize("skew", [False, True])
@pytest.mark.parametrize("euclid", [False, True])
def test_crel_gather_matches_per_item(skew, euclid, monkeypatch):
    """The rowtail gather's relation half as one [16 x R2] @ [R2 x d] MFMA product per tile
    (k_gather_crel: items in (row, type) order, per-(row, type) weight sums in LDS) against the
    per-item relation rows (REGCN_CREL_MIN_ITEMS=0): the same agg rows within 1e-5 * max|ref|
    (another fp32 association), on a snapshot whose leading tiles carry thousands of items;
    skew: one relation type takes 90 % of the edges, so (row, type) runs cross the waves' item
    ranges (the parked first runs).  Two runs are bitwise equal (no atomics)."""
    from regcn_amd import _lib
    from regcn_amd import graph as G
    from regcn_amd import hyperbolic_layers as HL
    V, R, d = 3000, 250, 200
    rng = np.random.default_rng(7)
    tr = _zipf_snapshot(V, R, 60000, 9)
    if skew:
        tr[:, 1] = np.where(rng.random(len(tr)) < 0.9, 3, tr[:, 1])
    g = G.build_sub_graph(V, R, tr, True, DEV, tile_budget=4096)
    wk = g.work()
    ip = wk["item_ptr"][:g.n_pos_tiles + 1].cpu().numpy()
    assert np.diff(ip).max() >= 2048
    gen = torch.Generator(device=DEV).manual_seed(3)
    x = (torch.randn(V, d, device=DEV, generator=gen) * 0.3).contiguous()
    r = (torch.rand(V, device=DEV, generator=gen) * 2.5 + 0.5).contiguous()
    rel = (torch.randn(2 * R, d, device=DEV, generator=gen) * 0.3).contiguous()
    mode = _lib.AGG_EUCLID if euclid else _lib.AGG_UNION
    w = torch.randn(d, d, device=DEV, generator=gen) * 0.05

    monkeypatch.setattr(HL, "CREL_MIN_TILES", 0)  # this snapshot has a handful of big tiles

    def gather(min_items):
        monkeypatch.setattr(HL, "CREL_MIN_ITEMS", min_items)
        g.__dict__.pop("_crel_tiles", None)
        agg = HL._heavy_aggregate(mode, g, x, r, rel, None, 1, 0.15, 0.01)
        if agg is None:
            agg = torch.zeros_like(x)
        h, xn, rn = HL._run_rowtail(mode, g, x, r, rel, None, 1, 0.15, w, w, w, 0.01, euclid, None, agg, None,
                                    None, int(wk["rows"].shape[0]))
        torch.cuda.synchronize()
        return agg.clone(), h.clone()

    a_ref, h_ref = gather(0)
    a1, h1 = gather(512)
    a2, h2 = gather(512)
    assert g.__dict__["_crel_tiles"][1] > 0
    rows = wk["rows"][:g.n_pos].long()
    ref = a_ref[rows]
    assert float((a1[rows] - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))
    assert torch.equal(a1, a2) and torch.equal(h1, h2)
    assert not torch.equal(a1[rows], ref)  # the product path ran (another fp32 association)
    assert float((h1 - h_ref).abs().max()) <= 1e-4


@pytest.mark.parametrize("c", [0.01, 0.05, 1.0])
def test_row_maps_fast_factor_math(c):
    """The row maps' factor math (common.h: v_sqrt / v_rcp / v_exp / v_log based tanh, atanh,
    norms and ratios) against float64 over row norms 1e-5 .. 30: within 2e-6 relative of the
    exact maps (the IEEE-library versions they replaced were within ~3e-7; parity needs 1e-4)."""
    from regcn_amd.hyperbolic_ops import HyperbolicOps as H
    g = torch.Generator().manual_seed(7)
    d = 200
    dirs = torch.nn.functional.normalize(torch.randn(4096, d, generator=g, dtype=torch.float64))
    norms = torch.logspace(-5, 1.5, 4096, dtype=torch.float64)[:, None]
    x = dirs * norms
    sc = c ** 0.5
    n = x.norm(dim=1, keepdim=True).clamp_min(1e-6)
    mx = 1 / sc - 2e-6  # project_to_ball's bound (hyperbolic_ops.py:37-74, eps twice)

    def project(y):
        ny = y.norm(dim=1, keepdim=True).clamp_min(1e-6)
        return y * torch.clamp(ny, max=mx) / ny

    exp_ref = project(torch.tanh(sc * n) * x / (sc * n))
    got = H.exp_map_zero(x.float().to(DEV), c).double().cpu()
    rel = ((got - exp_ref).norm(dim=1) / exp_ref.norm(dim=1)).max().item()
    assert rel <= 2e-6, "exp0 relative error %.3g" % rel
    xb = project(x * (0.9 / sc) / n.clamp_min(0.9 / sc))  # inside the ball
    nb = xb.norm(dim=1, keepdim=True).clamp_min(1e-6)
    log_ref = torch.atanh(torch.clamp(sc * nb, max=1 - 1e-6)) * xb / (sc * nb)
    got = H.log_map_zero(xb.float().to(DEV), c).double().cpu()
    rel = ((got - log_ref).norm(dim=1) / log_ref.norm(dim=1)).max().item()
    assert rel <= 2e-6, "log0 relative error %.3g" % rel
