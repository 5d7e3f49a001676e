"""Training path on the HIP kernels vs the reference's own loss values and
parameter gradients of one mini-batch (tests/golden/train_*.npz, made by running the
reference: tools/goldens/make_golden.py train), plus a few optimizer steps against the oracle.

Tolerance: losses 1e-4 relative; each gradient tensor |delta| <= 2e-3 max|ref| against the
reference's own fp32 run (its fp32 noise included), and <= 1e-4 max|ref| against the fp64 oracle
(test_training_grads_vs_fp64_oracle)."""
import numpy as np
import pytest
import torch

from regcn_amd import graph as G

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
C = 0.01

CASES = {
    "uvrgcn_roth": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False),
    "lgcn_roth": dict(encoder_name="lgcn", decoder_name="roth", layer_norm=False),
    "lgcn_roth_ln_skip": dict(encoder_name="lgcn", decoder_name="roth", layer_norm=True, skip_connect=True),
    "uvrgcn_murp_nores": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="murp", layer_norm=False,
                              use_residual_evolution=False),
    "uvrgcn_atth_beta": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="atth", layer_norm=True,
                             radius_anchor_beta=0.5),
    "uvrgcn_convtranse": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="hyperbolic_convtranse",
                              layer_norm=True),
    # the curvature features (tools/goldens/make_golden.py CURVATURE_TRAIN_CASES): a learned
    # curvature (grad of log_c through exp0 / log0 / mobius_add and the decoder scores) and the
    # per-relation curvature arctanh-distance score, alone and together
    "uvrgcn_roth_lc": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False,
                           learn_curvature=True),
    "lgcn_roth_crel_bias": dict(encoder_name="lgcn", decoder_name="roth", layer_norm=False,
                                use_relation_specific_curvature=True, use_entity_euclidean_bias=True),
    "uvrgcn_atth_lc_crel_ln": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="atth", layer_norm=True,
                                   learn_curvature=True, use_relation_specific_curvature=True),
}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def build(z, tag):
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    V, R, d, T = (int(v) for v in z["meta"])
    kw = dict(num_ents=V, num_rels=R, num_static_rels=0, num_words=0, h_dim=d, opn="sub", sequence_len=T,
              num_bases=d // 2, num_hidden_layers=2, dropout=0.0, c=C, self_loop=True, skip_connect=False,
              input_dropout=0.0, hidden_dropout=0.0, feat_dropout=0.0, entity_prediction=True,
              relation_prediction=True, use_cuda=True, gpu=0, radius_target=z["radius_target"],
              radius_msg_gamma=0.15)
    kw.update(CASES[tag])
    m = HyperbolicRecurrentRGCN(**kw)
    m.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd_")}, strict=True)
    m = m.to(DEV).train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            mod.eval()
    glist = [G.build_sub_graph(V, R, z["snap%d" % t], True, DEV) for t in range(T)]
    return m, glist


@pytest.mark.parametrize("tag", list(CASES))
def test_training_grads_vs_reference(golden, tag):
    z = golden("train_%s.npz" % tag)
    m, glist = build(z, tag)
    tw = float(z["task_weight"])
    le, lr, ls, lrad = m.get_loss(glist, torch.from_numpy(z["batch"]).to(DEV), None, True)
    loss = tw * le + (1 - tw) * lr + ls.sum() + lrad
    got = np.array([float(x.detach().sum()) for x in (le, lr, lrad, loss)])
    np.testing.assert_allclose(got, z["losses"][[0, 1, 3, 4]], rtol=1e-4, atol=1e-6)
    m.zero_grad()
    loss.backward()
    params = dict(m.named_parameters())
    n = 0
    for k in list(z):
        if not k.startswith("grad_"):
            continue
        g = params[k[5:]].grad
        assert g is not None, k
        ref = torch.from_numpy(z[k]).double()
        scale = max(1e-3, float(ref.abs().max()))
        err = float((g.detach().double().cpu() - ref).abs().max()) / scale
        assert err <= 2e-3, "%s: %.3g" % (k, err)
        n += 1
    assert n >= 20
    if "lc" in tag.split("_"):
        assert "grad_log_c" in z  # the learned curvature's gradient is among those checked


ORACLE_CFG = {
    "uvrgcn_roth": dict(encoder="hyperbolic_uvrgcn", decoder="roth", layer_norm=False),
    "lgcn_roth": dict(encoder="lgcn", decoder="roth", layer_norm=False),
    "lgcn_roth_ln_skip": dict(encoder="lgcn", decoder="roth", layer_norm=True, skip_connect=True),
    "uvrgcn_murp_nores": dict(encoder="hyperbolic_uvrgcn", decoder="murp", layer_norm=False,
                              use_residual_evolution=False),
    "uvrgcn_atth_beta": dict(encoder="hyperbolic_uvrgcn", decoder="atth", layer_norm=True, radius_anchor_beta=0.5),
    "uvrgcn_convtranse": dict(encoder="hyperbolic_uvrgcn", decoder="hyperbolic_convtranse", layer_norm=True),
}


def oracle_grads(z, tag, names):
    """fp64 gradients of the oracle's get_loss (oracle/model.py hyperbolic_get_loss, the
    reference op sequence) with respect to every parameter in `names`."""
    from oracle import graph as OG
    from oracle import model as OM
    V, R, d, T = (int(v) for v in z["meta"])
    sd = {k[3:]: torch.from_numpy(v).double() if v.dtype == np.float32 else torch.from_numpy(v)
          for k, v in z.items() if k.startswith("sd_")}
    for k in names:
        sd[k].requires_grad_(True)
    cfg = dict(c=C, n_layers=2, n_bases=d // 2, radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
               radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True)
    cfg.update(ORACLE_CFG[tag])
    og = [OG.build_sub_graph(V, R, z["snap%d" % t]) for t in range(T)]
    tw = float(z["task_weight"])
    le, lr, ls, lrad = OM.hyperbolic_get_loss(sd, cfg, og, torch.from_numpy(z["batch"]), z["radius_target"])
    (tw * le + (1 - tw) * lr + ls.sum() + lrad).backward()
    return {k: sd[k].grad for k in names}


@pytest.mark.parametrize("tag", list(ORACLE_CFG))
def test_training_grads_vs_fp64_oracle(golden, tag):
    """Every parameter gradient of one mini-batch against the fp64 oracle (the reference op
    sequence in double): |delta| <= 1e-4 * max(1e-3, max|ref|) per tensor (SURVEY.md §8(a)'s
    1e-4; the 2e-3 bound above is against the reference's own fp32 run, whose noise it
    includes)."""
    z = golden("train_%s.npz" % tag)
    m, glist = build(z, tag)
    tw = float(z["task_weight"])
    le, lr, ls, lrad = m.get_loss(glist, torch.from_numpy(z["batch"]).to(DEV), None, True)
    m.zero_grad()
    (tw * le + (1 - tw) * lr + ls.sum() + lrad).backward()
    params = dict(m.named_parameters())
    names = [k for k, p in params.items() if p.grad is not None]
    ref = oracle_grads(z, tag, names)
    worst = {}
    for k in names:
        if ref[k] is None:
            continue
        if k.endswith("score_margin") and float(ref[k].abs().max()) < 1e-12:
            # 0 analytically: the margin shifts every logit of a row alike, so the cross-entropy
            # gradient is scale * sum_b (sum_n softmax_bn - 1) / B; on the device it is the fp32
            # rounding of sum_n softmax (|delta| ~ 1e-7)
            assert float(params[k].grad.abs().max()) <= 1e-6, k
            continue
        scale = max(1e-3, float(ref[k].abs().max()))  # floor as above
        worst[k] = float((params[k].grad.double().cpu() - ref[k]).abs().max()) / scale
    bad = {k: v for k, v in worst.items() if v > 1e-4}
    assert not bad, "gradients over 1e-4 of max|ref|: %s" % bad
    print(tag, "worst gradient error vs fp64: %.3g (%s)" % max((v, k) for k, v in worst.items()))


def test_training_steps_vs_oracle(golden):
    """Three Adam steps (lr 1e-3, weight decay 1e-5, clip 1.0: hyperbolic_main.py:469, :627-628)
    on the lgcn+roth case: the HIP model and the oracle (fp64) keep the same loss trajectory."""
    from oracle import graph as OG
    from oracle import model as OM
    z = golden("train_lgcn_roth.npz")
    m, glist = build(z, "lgcn_roth")
    V, R, d, T = (int(v) for v in z["meta"])
    sd = {k[3:]: torch.from_numpy(v).double() if v.dtype == np.float32 else torch.from_numpy(v)
          for k, v in z.items() if k.startswith("sd_")}
    names = [k for k, _ in m.named_parameters()]
    oparams = [sd[k].requires_grad_(True) for k in names]
    cfg = dict(c=C, n_layers=2, n_bases=d // 2, radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
               radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True, encoder="lgcn",
               decoder="roth", layer_norm=False)
    og = [OG.build_sub_graph(V, R, z["snap%d" % t]) for t in range(T)]
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    oopt = torch.optim.Adam(oparams, lr=1e-3, weight_decay=1e-5)
    batch = torch.from_numpy(z["batch"])
    for step in range(3):
        opt.zero_grad()
        le, lr, ls, lrad = m.get_loss(glist, batch.to(DEV), None, True)
        loss = 0.7 * le + 0.3 * lr + ls.sum() + lrad
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        oopt.zero_grad()
        ole, olr, ols, olrad = OM.hyperbolic_get_loss(sd, cfg, og, batch, z["radius_target"])
        oloss = 0.7 * ole + 0.3 * olr + ols.sum() + olrad
        oloss.backward()
        torch.nn.utils.clip_grad_norm_(oparams, 1.0)
        oopt.step()
        assert abs(float(loss) - float(oloss)) <= 1e-4 * max(1.0, abs(float(oloss))), (step, float(loss), float(oloss))
    for k, p in zip(names, oparams):
        got = dict(m.named_parameters())[k].detach().double().cpu()
        assert float((got - p.detach()).abs().max()) <= 1e-4 * max(1.0, float(p.abs().max())), k


@pytest.mark.parametrize("tag", ["noln", "ln"])
def test_euclid_training_grads_vs_reference(golden, tag):
    """RecurrentRGCN.get_loss + backward (src/rrgcn.py:196-248; Euclidean RE-GCN, configs[0])."""
    from regcn_amd.rrgcn import RecurrentRGCN
    z = golden("train_rrgcn_%s.npz" % tag)
    V, R, d, T = (int(v) for v in z["meta"])
    m = RecurrentRGCN("convtranse", "uvrgcn", V, R, 0, 0, d, "sub", T, num_bases=100, num_basis=100,
                      num_hidden_layers=2, dropout=0.0, self_loop=True, skip_connect=False, layer_norm=(tag == "ln"),
                      input_dropout=0.0, hidden_dropout=0.0, feat_dropout=0.0, entity_prediction=True,
                      relation_prediction=True, use_cuda=True, gpu=0)
    m.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd_")}, strict=True)
    m = m.to(DEV).train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            mod.eval()
    glist = [G.build_sub_graph(V, R, z["snap%d" % t], True, DEV) for t in range(T)]
    tw = float(z["task_weight"])
    le, lr, ls = m.get_loss(glist, torch.from_numpy(z["batch"]).to(DEV), None, True)
    loss = tw * le + (1 - tw) * lr + ls.sum()
    got = np.array([float(x.detach().sum()) for x in (le, lr, loss)])
    np.testing.assert_allclose(got, z["losses"][[0, 1, 3]], rtol=1e-4, atol=1e-6)
    loss.backward()
    params = dict(m.named_parameters())
    n = 0
    for k in list(z):
        if k.startswith("grad_"):
            ref = torch.from_numpy(z[k]).double()
            g = params[k[5:]].grad
            err = float((g.detach().double().cpu() - ref).abs().max()) / max(1e-3, float(ref.abs().max()))
            assert err <= 2e-3, "%s: %.3g" % (k, err)
            n += 1
    assert n >= 15


@pytest.mark.parametrize("tag", ["lgcn_roth", "uvrgcn_convtranse"])
def test_encoder_reuse_same_gradients(golden, tag):
    """get_loss_batches (one encoder forward per snapshot, the CLI default) gives the
    gradients of hyperbolic_main.py:585-598's per-mini-batch get_loss + backward loop."""
    z = golden("train_%s.npz" % tag)
    batch = torch.from_numpy(z["batch"]).to(DEV)
    bs = max(1, batch.shape[0] // 3)
    m, glist = build(z, tag)
    m.zero_grad()
    for b in range(0, batch.shape[0], bs):
        le, lr, ls, lrad = m.get_loss(glist, batch[b:b + bs], None, True)
        (0.7 * le + 0.3 * lr + ls.sum() + lrad).backward()
    ref = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    m.zero_grad()
    parts = m.get_loss_batches(glist, batch, None, True, bs,
                               combine=lambda le, lr, ls, lrad: 0.7 * le + 0.3 * lr + ls.sum() + lrad)
    assert len(parts) == (batch.shape[0] + bs - 1) // bs
    assert all(not t.requires_grad for part in parts for t in part)  # backward already ran per mini-batch
    for k, p in m.named_parameters():
        if k in ref:
            err = float((p.grad - ref[k]).abs().max()) / max(1e-3, float(ref[k].abs().max()))
            assert err <= 1e-4, (k, err)


@pytest.mark.parametrize("learned_c,crel", [(True, False), (False, True)])
def test_loss_batches_memory_dense_fp64(learned_c, crel):
    """get_loss_batches' mini-batch groups on the dense fp64 decoder paths (a learned
    curvature's S matrix, the relation-specific curvature's arctanh-distance score) are sized
    for their fp64 B x N intermediates: at ICEWS18's |V| = 23,033 and batch 1024 one mini-batch
    per group (5 before), and the peak stays near one group's budgeted footprint."""
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    from regcn_amd.synthetic import zipf_triples
    V, R, d, bs = 23_033, 256, 64, 1024
    rng = np.random.default_rng(9)
    torch.manual_seed(9)
    m = HyperbolicRecurrentRGCN("roth", "hyperbolic_uvrgcn", V, R, 0, 0, d, "sub", 2, num_bases=d // 2,
                                num_hidden_layers=2, dropout=0.0, c=C, self_loop=True, entity_prediction=True,
                                relation_prediction=True, use_cuda=True, gpu=0, learn_curvature=learned_c,
                                use_relation_specific_curvature=crel).to(DEV).train()
    glist = [G.build_sub_graph(V, R, zipf_triples(rng, V, R, 20_000), True, DEV) for _ in range(2)]
    batch = torch.from_numpy(zipf_triples(rng, V, R, 4 * bs)).to(DEV)
    assert m._loss_group_size(bs, 1 << 28, learned_c) == 1
    assert m._loss_group_size(bs, 1 << 28, False) == (1 if crel else 5)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    parts = m.get_loss_batches(glist, batch, None, True, bs)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    assert len(parts) == 4
    one_group = 2 * bs * V * 4 * m.DENSE_FP64_WORDS  # the budgeted bytes of one mini-batch
    assert peak < 1.25 * one_group, "peak %.2f GB over one group's %.2f GB" % (peak / 2 ** 30, one_group / 2 ** 30)
