"""Dataset configs at their FULL shapes against the oracle (-m gpu): BASELINE.json configs[2]
(ICEWS18: |V| = 23,033, R = 256, ~1,540 triples per snapshot, history 3, hyperbolic_uvrgcn +
RotH) and configs[3] (GDELT: |V| = 7,691, R = 240, ~770 triples per snapshot, history 7, both
encoders), on the synthetic snapshots bench.py times (regcn_amd.synthetic) and the same
random-init weights (bench.build_model).

The HIP predict (the production dataset path: timestep phase launches, the fused RotH +
RotHRel decoder front) and oracle.model.hyperbolic_predict (the reference op sequence on the
CPU, hyperbolic_model.py:722-939) run on identical weights and snapshots.  Checked:
  * the last history embedding within 1e-4 * max(1, |ref|) on every row;
  * entity and relation scores within 1e-4 * max(1, |ref|);
  * per-query raw entity ranks equal except at near ties of the oracle's scores (a competitor
    within 1e-4 * max(1, |score|) of the target), and raw / time-filtered MRR (entity and
    relation) within the north star's 0.002.
The test queries are the first 256 triples of the next snapshot and their inverses (512 rows:
the CPU oracle scores 512 x |V| in seconds); the encoder runs the full snapshots."""
import pytest
import torch

from gpu_helpers import assert_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,encoder", [("icews18_roth", None), ("gdelt", None), ("gdelt", "lgcn")])
def test_dataset_full_shape_vs_oracle(name, encoder):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bench
    from oracle import graph as OG
    from oracle import model as OM
    from regcn_amd import graph as G
    from regcn_amd.synthetic import CONFIGS, snapshot_series
    cfg = dict(CONFIGS[name])
    if encoder:
        cfg["encoder"] = encoder
    V, R, T = cfg["V"], cfg["R"], cfg["T"]
    dev = torch.device("cuda", 0)
    snaps = snapshot_series(21, V, R, T + 1, cfg["per_snap"])
    model = bench.build_model(cfg, 200, dev, seed=3)
    test = snaps[T][:256]
    with torch.no_grad():
        glist = [G.build_sub_graph(V, R, s, True, dev) for s in snaps[:T]]
        assert glist[0].number_of_edges() == 2 * cfg["per_snap"]
        embs, _, _, _, _ = model.forward(glist, None, True)
        emb = embs[-1].float().cpu()
        all_tr, score, score_rel = model.predict(glist, R, None, torch.from_numpy(test).to(dev), True)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    ocfg = dict(c=0.01, n_layers=2, n_bases=cfg["n_bases"], radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
                radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True, layer_norm=False,
                encoder=cfg["encoder"], decoder=cfg["decoder"])
    og = [OG.build_sub_graph(V, R, s) for s in snaps[:T]]
    o_tr, o_score, o_score_rel, o_embs, _ = OM.hyperbolic_predict(sd, ocfg, og, torch.from_numpy(test))
    assert torch.equal(all_tr.cpu(), o_tr)
    assert_close(emb, o_embs[-1], what="%s last history embedding" % name)
    assert_close(score.cpu(), o_score, what="%s entity scores" % name)
    assert_close(score_rel.cpu(), o_score_rel, what="%s relation scores" % name)
    ans_e = OM.answers_for_filter(snaps[T], R)
    ans_r = OM.answers_for_filter(snaps[T], R, True)
    mrr = {}
    ranks = {}
    for pre, sc, sr in (("hip", score.float().cpu(), score_rel.float().cpu()), ("or", o_score, o_score_rel)):
        _, _, r_e, f_e = OM.total_rank(o_tr, sc, ans_e)
        _, _, r_r, f_r = OM.total_rank(o_tr, sr, ans_r, True)
        ranks[pre] = r_e
        for k, v in (("re", r_e), ("fe", f_e), ("rr", r_r), ("fr", f_r)):
            mrr[pre + "_" + k] = float(torch.mean(1.0 / v.float()))
    diff = (ranks["hip"] - ranks["or"]).abs()
    tgt = o_score.gather(1, o_tr[:, 2:3].long())
    close = ((o_score - tgt).abs() <= 1e-4 * torch.clamp(tgt.abs(), min=1.0)).sum(1) - 1
    assert bool((diff <= close).all()), "entity rank differences without a near tie"
    for k in ("re", "fe", "rr", "fr"):
        assert abs(mrr["hip_" + k] - mrr["or_" + k]) <= 0.002, (k, mrr)
    print(name, encoder or cfg["encoder"], {k: round(v, 5) for k, v in mrr.items()},
          "rank flips at near ties: %d of %d" % (int((diff > 0).sum()), diff.numel()))


def test_regcn_icews14s_full_shape_vs_oracle():
    """BASELINE.json configs[0] at its real shape: the Euclidean RE-GCN (RecurrentRGCN +
    ConvTransE / ConvTransR, src/rrgcn.py:142-194, src/decoder.py:10-100) with the reference's
    ICEWS14s command (d = 200, 2 layers, self-loop, layer norm, history 3) on ICEWS14s-shaped
    snapshots (|V| = 7,128, R = 230, 246 triples each) against oracle.model.euclid_predict on the
    same random-init weights: every history embedding, h_0 and both decoders' scores within
    1e-4 * max(1, |ref|); entity ranks equal up to near ties; MRRs within 0.002."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from oracle import graph as OG
    from oracle import model as OM
    from regcn_amd import graph as G
    from regcn_amd.rrgcn import RecurrentRGCN
    from regcn_amd.synthetic import CONFIGS, snapshot_series
    cfg = CONFIGS["icews14s_uvrgcn_convtranse"]
    V, R, T, d = cfg["V"], cfg["R"], cfg["T"], 200
    dev = torch.device("cuda", 0)
    snaps = snapshot_series(23, V, R, T + 1, cfg["per_snap"])
    torch.manual_seed(4)
    m = RecurrentRGCN("convtranse", "uvrgcn", V, R, 0, 0, d, "sub", T, num_bases=100, num_basis=100,
                      num_hidden_layers=2, dropout=0.2, self_loop=True, layer_norm=True, input_dropout=0.2,
                      hidden_dropout=0.2, feat_dropout=0.2, entity_prediction=True, relation_prediction=True,
                      use_cuda=True, gpu=0)
    with torch.no_grad():  # non-trivial batch-norm statistics for the eval-mode decoders
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
    m = m.to(dev).eval()
    test = snaps[T]
    with torch.no_grad():
        glist = [G.build_sub_graph(V, R, s, True, dev) for s in snaps[:T]]
        assert glist[0].number_of_edges() == 2 * cfg["per_snap"]
        embs, _, h0, _, _ = m.forward(glist, None, True)
        all_tr, score, score_rel = m.predict(glist, R, None, torch.from_numpy(test).to(dev), True)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    og = [OG.build_sub_graph(V, R, s) for s in snaps[:T]]
    o_tr, o_score, o_score_rel, o_embs, o_h0 = OM.euclid_predict(sd, dict(layer_norm=True, n_layers=2), og,
                                                                  torch.from_numpy(test))
    assert torch.equal(all_tr.cpu(), o_tr)
    for t in range(T):
        assert_close(embs[t].cpu(), o_embs[t], what="history embedding %d" % t)
    assert_close(h0.cpu(), o_h0, what="h_0")
    assert_close(score.cpu(), o_score, what="ConvTransE scores")
    assert_close(score_rel.cpu(), o_score_rel, what="ConvTransR scores")
    ans_e = OM.answers_for_filter(test, R)
    ans_r = OM.answers_for_filter(test, R, True)
    mrr, ranks = {}, {}
    for pre, sc, sr in (("hip", score.float().cpu(), score_rel.float().cpu()), ("or", o_score, o_score_rel)):
        _, _, r_e, f_e = OM.total_rank(o_tr, sc, ans_e)
        _, _, r_r, f_r = OM.total_rank(o_tr, sr, ans_r, True)
        ranks[pre] = r_e
        for k, v in (("re", r_e), ("fe", f_e), ("rr", r_r), ("fr", f_r)):
            mrr[pre + "_" + k] = float(torch.mean(1.0 / v.float()))
    diff = (ranks["hip"] - ranks["or"]).abs()
    tgt = o_score.gather(1, o_tr[:, 2:3].long())
    close = ((o_score - tgt).abs() <= 1e-4 * torch.clamp(tgt.abs(), min=1.0)).sum(1) - 1
    assert bool((diff <= close).all()), "entity rank differences without a near tie"
    for k in ("re", "fe", "rr", "fr"):
        assert abs(mrr["hip_" + k] - mrr["or_" + k]) <= 0.002, (k, mrr)
