"""Generate golden input/output vectors by running the REFERENCE code on CPU.

CONTAINER ONLY.  This script imports the read-only reference tree at
/root/reference (through the test-only DGL stand-in in ./standin) and writes
small .npz fixtures into tests/golden/.  The fixtures are data (inputs and the
reference's outputs); no reference source travels with them.  Nothing on the
GPU box runs this script.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/goldens/make_golden.py

Each fixture pins one row of SURVEY.md §8(a):
  graph_indexing.npz   a1  build_sub_graph + r2e           rgcn/utils.py:78-134
  ops.npz              a3  HyperbolicOps / LorentzOps        hyperbolic_ops.py:37-233, 476-581
  layer_union.npz      a4  HyperbolicUnionRGCNLayer          hyperbolic_layers.py:164-323
  layer_euclid.npz     a5  UnionRGCNLayer                    rgcn/layers.py:182-279
  layer_lorentz.npz    a6  LorentzRGCNLayer                  hyperbolic_layers.py:524-694
  model_*.npz          a9  HyperbolicRecurrentRGCN.predict / get_loss   hyperbolic_model.py:722-1088
                           (models_large: d = 200 at the ICEWS18 / GDELT shapes, predict only)
  rrgcn_*.npz          a9  RecurrentRGCN.predict             src/rrgcn.py:142-194
                           (rrgcn_ln_d200: d = 200 at ICEWS14s' R = 230; "rrgcn_large")
  score.npz            a11/a12 chunked dist score / CE       hyperbolic_decoder.py:89-307
  rank.npz             f2  get_total_rank / filter_score     rgcn/utils.py:21-166
  multistep.npz        f2  filtered scores left by get_total_rank -> construct_snap(_r)
                           (the --multi-step history roll)   rgcn/utils.py:51-75, 367-405;
                                                             hyperbolic_main.py:116-149
  train_*.npz          f1  get_loss + backward: every parameter gradient   hyperbolic_main.py:585-598
  analysis_*.npz       N1  --run-analysis: gate_list, time-gate means, radius-evolution stats,
                           embedding stats, loss components, gradient norm, training summary
                                                             hyperbolic_model.py:747-890, :1076-1127;
                                                             hyperbolic_ops.py:235-269, :426-439
  tkg_tiny/ + dataset_tiny.npz  f4  load_from_local + split_by_time on a dataset directory
                                                             knowledge_graph.py:189-206, 526-555;
                                                             rgcn/utils.py:306-339
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "standin"))
sys.path.insert(0, REF)

# rgcn/layers.py:229-231 calls .cuda() unconditionally; make it a no-op on CPU.
torch.Tensor.cuda = lambda self, *a, **k: self  # noqa: E731

from rgcn import utils as rutils  # noqa: E402
from rgcn.layers import UnionRGCNLayer  # noqa: E402
from hyperbolic_src.hyperbolic_ops import HyperbolicOps, LorentzOps  # noqa: E402
from hyperbolic_src.hyperbolic_layers import HyperbolicUnionRGCNLayer, LorentzRGCNLayer  # noqa: E402
from hyperbolic_src import hyperbolic_decoder as hdec  # noqa: E402
from hyperbolic_src.hyperbolic_model import HyperbolicRecurrentRGCN  # noqa: E402
from src.rrgcn import RecurrentRGCN  # noqa: E402
import torch.nn.functional as F  # noqa: E402

C = 0.01


def zipf_triples(rng, V, R, T, alpha=1.1, self_loops=0, dups=0):
    perm = rng.permutation(V)
    p = 1.0 / np.arange(1, V + 1) ** alpha
    p /= p.sum()
    s = perm[rng.choice(V, size=T, p=p)]
    o = perm[rng.choice(V, size=T, p=p)]
    r = rng.integers(0, R, size=T)
    tr = np.stack([s, r, o], 1).astype(np.int64)
    if self_loops:
        tr[:self_loops, 2] = tr[:self_loops, 0]
    if dups:
        tr[-dups:] = tr[self_loops:self_loops + dups]
    return tr


def ball_points(gen, n, d, rmin=0.5, rmax=3.0):
    x = HyperbolicOps.exp_map_zero(torch.randn(n, d, generator=gen), C)
    rad = rmin + (rmax - rmin) * torch.rand(n, generator=gen)
    return HyperbolicOps.apply_radius(x, rad, C)


def graph_arrays(g, prefix=""):
    return {
        prefix + "src": g._src.numpy(), prefix + "dst": g._dst.numpy(),
        prefix + "type": g.edata["type"].numpy(),
        prefix + "in_deg": g.in_degrees(range(g.number_of_nodes())).numpy(),
        prefix + "norm": g.ndata["norm"].numpy().reshape(-1),
        prefix + "enorm": g.edata["norm"].numpy().reshape(-1),
        prefix + "uniq_r": np.asarray(g.uniq_r), prefix + "r_len": np.asarray(g.r_len).reshape(-1, 2),
        prefix + "r_to_e": np.asarray(g.r_to_e, dtype=np.int64),
    }


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote", path, "%.0f KB" % (os.path.getsize(path) / 1024))


def gen_graph_indexing():
    rng = np.random.default_rng(1)
    out = {}
    cases = [("small", 64, 8, 200, 6, 10), ("mid", 500, 40, 3000, 20, 50), ("empty_rel", 30, 12, 40, 2, 3)]
    for tag, V, R, T, sl, dup in cases:
        tr = zipf_triples(rng, V, R, T, self_loops=sl, dups=dup)
        if tag == "empty_rel":
            tr[:, 1] = tr[:, 1] % 5 * 2  # only even relation ids < 10 present
        g = rutils.build_sub_graph(V, R, tr, False, "cpu")
        out[tag + "_triples"] = tr
        out[tag + "_meta"] = np.array([V, R])
        out.update(graph_arrays(g, tag + "_"))
    save("graph_indexing.npz", **out)


def gen_ops():
    gen = torch.Generator().manual_seed(2)
    d = 200
    out = {}
    for cname, c in (("c01", 0.01), ("c05", 0.05)):
        base = torch.randn(16, d, generator=gen)
        unit = base / base.norm(dim=-1, keepdim=True)
        bound = 1.0 / np.sqrt(c)
        norms = torch.tensor([0.0, 1e-9, 1e-5, 1e-3, 0.1, 1.0, 3.0, 0.5 * bound, 0.9 * bound,
                              0.99 * bound, 0.9999 * bound, bound - 1e-6, bound, bound + 1e-3,
                              1.5 * bound, 0.2], dtype=torch.float32)
        x = unit * norms[:, None]
        x[0] = 0.0
        v = unit * torch.tensor([0.0, 1e-8, 1e-4, 0.01, 1.0, 5.0, 10.0, 20.0, 50.0, 80.0, 100.0,
                                 200.0, 1e3, 1e4, 3.0, 0.3], dtype=torch.float32)[:, None]
        y = ball_points(gen, 16, d) * (1.0 if c == 0.01 else 0.4)
        rad = torch.tensor([1e-8, 0.5, 1.0, 2.0, 3.0, 5.0, 9.0, 9.999999, 10.0, 11.0, 20.0, 0.7,
                            1.3, 2.2, 4.4, 6.0], dtype=torch.float32)
        out[cname + "_x"] = x.numpy()
        out[cname + "_v"] = v.numpy()
        out[cname + "_y"] = y.numpy()
        out[cname + "_rad"] = rad.numpy()
        out[cname + "_project"] = HyperbolicOps.project_to_ball(x, c).numpy()
        out[cname + "_log0"] = HyperbolicOps.log_map_zero(x, c).numpy()
        out[cname + "_exp0"] = HyperbolicOps.exp_map_zero(v, c).numpy()
        xb = HyperbolicOps.project_to_ball(x, c)
        out[cname + "_mobius"] = HyperbolicOps.mobius_add(xb, y, c).numpy()
        out[cname + "_dist"] = HyperbolicOps.hyperbolic_distance(xb, y, c).numpy()
        out[cname + "_radius"] = HyperbolicOps.get_radius(x).numpy()
        out[cname + "_apply_radius"] = HyperbolicOps.apply_radius(y, rad, c).numpy()
        L = LorentzOps.to_lorentz(y, c)
        out[cname + "_to_lorentz"] = L.numpy()
        out[cname + "_to_poincare"] = LorentzOps.to_poincare(L, c).numpy()
        w = torch.rand(16, generator=gen)
        out[cname + "_w"] = w.numpy()
        out[cname + "_centroid"] = LorentzOps.lorentz_centroid(L, w, c).numpy()
    save("ops.npz", **out)


def layer_graph(seed, V=300, R=256, T=1000, d=200, zero_deg_min=40):
    rng = np.random.default_rng(seed)
    tr = zipf_triples(rng, V, R, T, self_loops=5, dups=20)
    g = rutils.build_sub_graph(V, R, tr, False, "cpu")
    deg = g.in_degrees(range(V)).numpy()
    assert (deg == 0).sum() >= zero_deg_min, (deg == 0).sum()
    return tr, g


def gen_layer_union():
    torch.manual_seed(3)
    gen = torch.Generator().manual_seed(3)
    V, R, d = 300, 128, 200
    tr, g = layer_graph(3, V, R, 1000, d)
    h = ball_points(gen, V, d)
    prev = ball_points(gen, V, d)
    rel = torch.randn(2 * R, d, generator=gen) * 0.3
    out = {"triples": tr, "meta": np.array([V, R, d]), "h": h.numpy(), "prev_h": prev.numpy(),
           "rel": rel.numpy()}
    shared = None
    for gname, gamma in (("g0", 0.0), ("g15", 0.15)):
        for skip in (False, True):
            lay = HyperbolicUnionRGCNLayer(d, d, 2 * R, -1, c=C, activation=F.rrelu, self_loop=True,
                                           dropout=0.2, skip_connect=skip, radius_msg_gamma=gamma)
            if shared is None:
                shared = {k: v.clone() for k, v in lay.state_dict().items()}
                for k, v in shared.items():
                    out["w_" + k] = v.numpy()
            if skip and "w_skip_weight" not in out:
                out["w_skip_weight"] = lay.skip_weight.detach().numpy()
                out["w_skip_bias"] = (torch.randn(d, generator=gen) * 0.1).numpy()
            sd = {k: torch.from_numpy(out["w_" + k]) for k in lay.state_dict()}
            lay.load_state_dict(sd)
            lay.eval()
            with torch.no_grad():
                y = lay(g, h, rel, prev_h=prev if skip else None)
            out["%s_%s_out" % (gname, "skip" if skip else "noskip")] = y.numpy()
    save("layer_union.npz", **out)


def gen_layer_euclid():
    torch.manual_seed(4)
    gen = torch.Generator().manual_seed(4)
    V, R, d = 300, 256, 200
    tr, g = layer_graph(4, V, R, 1000, d)
    h = torch.randn(V, d, generator=gen) * 0.5
    rel = torch.randn(2 * R, d, generator=gen) * 0.3
    out = {"triples": tr, "meta": np.array([V, R, d]), "h": h.numpy(), "rel": rel.numpy()}
    lay = UnionRGCNLayer(d, d, 2 * R, -1, activation=F.rrelu, self_loop=True, dropout=0.2)
    lay.eval()
    g.ndata["h"] = h
    with torch.no_grad():
        y = lay(g, [], rel)
    out["out"] = y.numpy()
    for k, v in lay.state_dict().items():
        out["w_" + k] = v.numpy()
    save("layer_euclid.npz", **out)


def gen_layer_lorentz():
    out = {}
    # (tag, d, R, n_bases) -> submatrix s = d / min(n_bases, 2R)
    cases = [("s2", 200, 64, 100), ("s4", 64, 32, 16), ("s1", 64, 32, 64), ("s20", 60, 16, 3)]
    for i, (tag, d, R, nb) in enumerate(cases):
        torch.manual_seed(10 + i)
        gen = torch.Generator().manual_seed(10 + i)
        V = 300
        tr, g = layer_graph(10 + i, V, R, 1000, d)
        h = ball_points(gen, V, d)
        prev = ball_points(gen, V, d)
        rel = torch.randn(2 * R, d, generator=gen) * 0.3
        out[tag + "_triples"] = tr
        out[tag + "_meta"] = np.array([V, R, d, nb])
        out[tag + "_h"] = h.numpy()
        out[tag + "_prev_h"] = prev.numpy()
        out[tag + "_rel"] = rel.numpy()
        for skip in ((False, True) if tag == "s2" else (False,)):
            lay = LorentzRGCNLayer(d, d, 2 * R, nb, c=C, activation=F.rrelu, self_loop=True,
                                   dropout=0.2, skip_connect=skip)
            for k, v in lay.state_dict().items():
                if tag + "_w_" + k not in out:
                    out[tag + "_w_" + k] = v.numpy()
            if skip:
                out[tag + "_w_skip_bias"] = (torch.randn(d, generator=gen) * 0.1).numpy()
            lay.load_state_dict({k: torch.from_numpy(out[tag + "_w_" + k]) for k in lay.state_dict()})
            lay.eval()
            with torch.no_grad():
                y = lay(g, h, rel, prev_h=prev if skip else None)
            out[tag + ("_skip" if skip else "_noskip") + "_out"] = y.numpy()
    save("layer_lorentz.npz", **out)


def snapshot_series(seed, V, R, n_snap, per_snap):
    """Synthetic TKG snapshots with temporal recurrence."""
    rng = np.random.default_rng(seed)
    snaps = []
    for t in range(n_snap):
        tr = zipf_triples(rng, V, R, per_snap)
        if snaps:
            k = int(0.6 * per_snap)
            pool = np.concatenate(snaps[-3:])
            tr[:k] = pool[rng.integers(0, len(pool), size=k)]
        snaps.append(tr)
    return snaps


def gen_models():
    V, R, T = 256, 64, 3
    snaps = snapshot_series(20, V, R, T + 1, 120)
    rng = np.random.default_rng(21)
    radius_target = rng.uniform(0.5, 3.0, size=V).astype(np.float32)
    cases = [
        ("uvrgcn_roth", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False)),
        ("uvrgcn_roth_ln", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=True)),
        ("lgcn_roth", dict(encoder_name="lgcn", decoder_name="roth", layer_norm=False)),
        ("lgcn_roth_ln", dict(encoder_name="lgcn", decoder_name="roth", layer_norm=True)),
        ("uvrgcn_murp_nores", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="murp", layer_norm=False,
                                   use_residual_evolution=False)),
        ("uvrgcn_atth_beta", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="atth", layer_norm=True,
                                  radius_anchor_beta=0.5)),
        ("lgcn_roth_bias_crel", dict(encoder_name="lgcn", decoder_name="roth", layer_norm=False,
                                     use_entity_euclidean_bias=True, use_relation_specific_curvature=True)),
        ("uvrgcn_convtranse", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="hyperbolic_convtranse",
                                   layer_norm=True)),
    ]
    glist = [rutils.build_sub_graph(V, R, s, False, "cpu") for s in snaps[:T]]
    test = torch.from_numpy(snaps[T])
    for i, (tag, kw) in enumerate(cases):
        torch.manual_seed(100 + i)
        # d=200 (the north-star width) for the configs[1] encoder/decoder pair, d=64 elsewhere to keep the
        # fixtures small; n_bases gives 2x2 Lorentz blocks in both.
        d = 200 if tag == "lgcn_roth" else 64
        base = dict(num_ents=V, num_rels=R, num_static_rels=0, num_words=0, h_dim=d, opn="sub",
                    sequence_len=T, num_bases=d // 2, num_hidden_layers=2, dropout=0.2, c=C,
                    self_loop=True, skip_connect=False, input_dropout=0.2, hidden_dropout=0.2,
                    feat_dropout=0.2, entity_prediction=True, relation_prediction=True,
                    use_cuda=False, gpu="cpu", radius_target=radius_target, radius_msg_gamma=0.15)
        base.update(kw)
        m = HyperbolicRecurrentRGCN(**base)
        with torch.no_grad():
            # make the decoder scales/biases non-trivial so the epilogue is exercised
            for mod in (m.decoder_ob, m.rdecoder):
                if hasattr(mod, "score_margin"):
                    mod.score_margin.fill_(0.7)
                    mod.score_scale_raw.fill_(0.4)
                if getattr(mod, "entity_bias", None) is not None:
                    mod.entity_bias.normal_(0, 0.1)
                if getattr(mod, "rel_bias", None) is not None:
                    mod.rel_bias.normal_(0, 0.1)
            m.radius_static.add_(torch.randn(V) * 0.2)
        m.eval()
        with torch.no_grad():
            embs, _, h0, _, _ = m.forward(glist, None, False)
            all_tr, score, score_rel = m.predict(glist, R, None, test.clone(), False)
        out = {"meta": np.array([V, R, d, T]), "test": snaps[T], "all_triples": all_tr.numpy(),
               "score": score.numpy(), "score_rel": score_rel.numpy(), "h0": h0.numpy(),
               "embs": torch.stack(embs).numpy(), "radius_target": radius_target}
        for t in range(T):
            out["snap%d" % t] = snaps[t]
        for k, v in m.state_dict().items():
            out["sd_" + k] = v.numpy().copy()
        # deterministic loss: model.train() but every dropout p=0 and BatchNorm frozen
        m.train()
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.eval()
        losses = m.get_loss(glist, test.clone(), None, False)
        out["losses"] = np.array([x.item() for x in losses])
        save("model_%s.npz" % tag, **out)


# Dataset-shaped model goldens at d = 200: the ICEWS18 relation
# count (R2 = 512) with hub rows over the fused kernel's inline budget, the same at |E| = 80k
# (the large-snapshot work lists: short chunks, small budget, many pre-aggregated rows), and
# the GDELT history length 7 for both encoders.  Only the last history embedding is stored.
LARGE_CASES = [
    ("uvrgcn_roth_r512_d200", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False),
     dict(V=1536, R=256, T=3, per_snap=2500, n_test=64, seed=50)),
    ("uvrgcn_roth_e80k_d200", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False),
     dict(V=2048, R=256, T=3, per_snap=40000, n_test=64, seed=51)),
    ("uvrgcn_roth_h7_d200", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False),
     dict(V=1024, R=240, T=7, per_snap=770, n_test=128, seed=52)),
    ("lgcn_roth_h7_d200", dict(encoder_name="lgcn", decoder_name="roth", layer_norm=True),
     dict(V=1024, R=240, T=7, per_snap=770, n_test=128, seed=53)),
]


def gen_models_large():
    d = 200
    for i, (tag, kw, sz) in enumerate(LARGE_CASES):
        V, R, T = sz["V"], sz["R"], sz["T"]
        snaps = snapshot_series(sz["seed"], V, R, T + 1, sz["per_snap"])
        rng = np.random.default_rng(sz["seed"] + 100)
        radius_target = rng.uniform(0.5, 3.0, size=V).astype(np.float32)
        glist = [rutils.build_sub_graph(V, R, s, False, "cpu") for s in snaps[:T]]
        test_np = snaps[T][:sz["n_test"]]
        test = torch.from_numpy(test_np)
        torch.manual_seed(500 + i)
        base = dict(num_ents=V, num_rels=R, num_static_rels=0, num_words=0, h_dim=d, opn="sub",
                    sequence_len=T, num_bases=d // 2, num_hidden_layers=2, dropout=0.2, c=C,
                    self_loop=True, skip_connect=False, input_dropout=0.2, hidden_dropout=0.2,
                    feat_dropout=0.2, entity_prediction=True, relation_prediction=True,
                    use_cuda=False, gpu="cpu", radius_target=radius_target, radius_msg_gamma=0.15)
        base.update(kw)
        m = HyperbolicRecurrentRGCN(**base)
        with torch.no_grad():
            for mod in (m.decoder_ob, m.rdecoder):
                if hasattr(mod, "score_margin"):
                    mod.score_margin.fill_(0.7)
                    mod.score_scale_raw.fill_(0.4)
                if getattr(mod, "rel_bias", None) is not None:
                    mod.rel_bias.normal_(0, 0.1)
            m.radius_static.add_(torch.randn(V) * 0.2)
        m.eval()
        with torch.no_grad():
            embs, _, h0, _, _ = m.forward(glist, None, False)
            all_tr, score, score_rel = m.predict(glist, R, None, test.clone(), False)
        out = {"meta": np.array([V, R, d, T]), "test": test_np, "all_triples": all_tr.numpy(),
               "score": score.numpy(), "score_rel": score_rel.numpy(), "h0": h0.numpy(),
               "embs_last": embs[-1].numpy(), "radius_target": radius_target}
        for t in range(T):
            out["snap%d" % t] = snaps[t].astype(np.int32)  # ids < 2^31: half the fixture
        for k, v in m.state_dict().items():
            out["sd_" + k] = v.numpy().copy()
        save("model_%s.npz" % tag, **out)


TRAIN_CASES = [
    ("uvrgcn_roth", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False)),
    ("lgcn_roth", dict(encoder_name="lgcn", decoder_name="roth", layer_norm=False)),
    ("lgcn_roth_ln_skip", dict(encoder_name="lgcn", decoder_name="roth", layer_norm=True, skip_connect=True)),
    ("uvrgcn_murp_nores", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="murp", layer_norm=False,
                               use_residual_evolution=False)),
    ("uvrgcn_atth_beta", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="atth", layer_norm=True,
                              radius_anchor_beta=0.5)),
    ("uvrgcn_convtranse", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="hyperbolic_convtranse",
                               layer_norm=True)),
]


CURVATURE_TRAIN_CASES = [
    ("uvrgcn_roth_lc", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False,
                            learn_curvature=True)),
    ("lgcn_roth_crel_bias", dict(encoder_name="lgcn", decoder_name="roth", layer_norm=False,
                                 use_relation_specific_curvature=True, use_entity_euclidean_bias=True)),
    ("uvrgcn_atth_lc_crel_ln", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="atth", layer_norm=True,
                                    learn_curvature=True, use_relation_specific_curvature=True)),
]


def gen_train_curvature():
    """gen_train's mini-batch for the two curvature features whose gradients the build adds
    this round: a learned curvature (log_c, hyperbolic_model.py:299-300, :673-679, :753-770)
    and the per-relation curvature arctanh-distance score (hyperbolic_decoder.py:145-164,
    :257-283), alone and together."""
    V, R, T, d, tw = 256, 64, 3, 64, 0.7
    snaps = snapshot_series(40, V, R, T + 1, 120)
    rng = np.random.default_rng(41)
    radius_target = rng.uniform(0.5, 3.0, size=V).astype(np.float32)
    glist = [rutils.build_sub_graph(V, R, s, False, "cpu") for s in snaps[:T]]
    batch = torch.from_numpy(snaps[T])
    for i, (tag, kw) in enumerate(CURVATURE_TRAIN_CASES):
        torch.manual_seed(350 + i)
        base = dict(num_ents=V, num_rels=R, num_static_rels=0, num_words=0, h_dim=d, opn="sub",
                    sequence_len=T, num_bases=d // 2, num_hidden_layers=2, dropout=0.0, c=C,
                    self_loop=True, skip_connect=False, input_dropout=0.0, hidden_dropout=0.0,
                    feat_dropout=0.0, entity_prediction=True, relation_prediction=True,
                    use_cuda=False, gpu="cpu", radius_target=radius_target, radius_msg_gamma=0.15)
        base.update(kw)
        m = HyperbolicRecurrentRGCN(**base)
        with torch.no_grad():
            for mod in (m.decoder_ob, m.rdecoder):
                if hasattr(mod, "score_margin"):
                    mod.score_margin.fill_(0.7)
                    mod.score_scale_raw.fill_(0.4)
                if getattr(mod, "rel_bias", None) is not None:
                    mod.rel_bias.normal_(0, 0.1)
                if getattr(mod, "entity_bias", None) is not None:
                    mod.entity_bias.normal_(0, 0.1)
                if getattr(mod, "rel_curvature_raw", None) is not None:  # spread the curvatures
                    mod.rel_curvature_raw.add_(torch.randn(mod.rel_curvature_raw.shape) * 0.5)
                for lin in mod.modules():
                    if isinstance(lin, torch.nn.Linear) and lin.weight.shape[0] == lin.weight.shape[1]:
                        lin.weight.normal_(0, 0.05)
            m.radius_static.add_(torch.randn(V) * 0.2)
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        m.train()
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.eval()
        m.zero_grad()
        le, lr, ls, lrad = m.get_loss(glist, batch.clone(), None, False)
        loss = tw * le + (1 - tw) * lr + ls + lrad
        loss.backward()
        out = {"meta": np.array([V, R, d, T]), "batch": snaps[T], "radius_target": radius_target,
               "task_weight": np.array(tw), "losses": np.array([float(x) for x in (le, lr, ls, lrad, loss)])}
        for t in range(T):
            out["snap%d" % t] = snaps[t]
        for k, v in sd.items():
            out["sd_" + k] = v.numpy().copy()
        for k, p in m.named_parameters():
            if p.grad is not None:
                out["grad_" + k] = p.grad.numpy().copy()
        save("train_%s.npz" % tag, **out)


def gen_train():
    """One training mini-batch (hyperbolic_main.py:585-598): get_loss on the snapshot's triples,
    loss = tw le + (1 - tw) lr + ls + lrad, backward; every parameter's gradient.  Dropout p = 0
    and BatchNorm frozen so the step is deterministic."""
    V, R, T, d, tw = 256, 64, 3, 64, 0.7
    snaps = snapshot_series(40, V, R, T + 1, 120)
    rng = np.random.default_rng(41)
    radius_target = rng.uniform(0.5, 3.0, size=V).astype(np.float32)
    glist = [rutils.build_sub_graph(V, R, s, False, "cpu") for s in snaps[:T]]
    batch = torch.from_numpy(snaps[T])
    for i, (tag, kw) in enumerate(TRAIN_CASES):
        torch.manual_seed(300 + i)
        base = dict(num_ents=V, num_rels=R, num_static_rels=0, num_words=0, h_dim=d, opn="sub",
                    sequence_len=T, num_bases=d // 2, num_hidden_layers=2, dropout=0.0, c=C,
                    self_loop=True, skip_connect=False, input_dropout=0.0, hidden_dropout=0.0,
                    feat_dropout=0.0, entity_prediction=True, relation_prediction=True,
                    use_cuda=False, gpu="cpu", radius_target=radius_target, radius_msg_gamma=0.15)
        base.update(kw)
        m = HyperbolicRecurrentRGCN(**base)
        with torch.no_grad():
            for mod in (m.decoder_ob, m.rdecoder):
                if hasattr(mod, "score_margin"):
                    mod.score_margin.fill_(0.7)
                    mod.score_scale_raw.fill_(0.4)
                if getattr(mod, "rel_bias", None) is not None:
                    mod.rel_bias.normal_(0, 0.1)
                for lin in mod.modules():  # the 1e-3 init makes the decoder MLPs near-identity
                    if isinstance(lin, torch.nn.Linear) and lin.weight.shape[0] == lin.weight.shape[1]:
                        lin.weight.normal_(0, 0.05)
            m.radius_static.add_(torch.randn(V) * 0.2)
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        m.train()
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.eval()
        m.zero_grad()
        le, lr, ls, lrad = m.get_loss(glist, batch.clone(), None, False)
        loss = tw * le + (1 - tw) * lr + ls + lrad
        loss.backward()
        out = {"meta": np.array([V, R, d, T]), "batch": snaps[T], "radius_target": radius_target,
               "task_weight": np.array(tw), "losses": np.array([float(x) for x in (le, lr, ls, lrad, loss)])}
        for t in range(T):
            out["snap%d" % t] = snaps[t]
        for k, v in sd.items():
            out["sd_" + k] = v.numpy().copy()
        for k, p in m.named_parameters():
            if p.grad is not None:
                out["grad_" + k] = p.grad.numpy().copy()
        save("train_%s.npz" % tag, **out)
    # Euclidean RE-GCN (src/rrgcn.py:196-248, src/main.py's loss).  Its CPU branch adds in place
    # to a leaf zeros(1, requires_grad=True) and raises; on the GPU branch `.cuda()` returns a
    # non-leaf copy.  Emulate that branch: use_cuda=True with .cuda() a copy on the CPU.
    torch.Tensor.cuda = lambda self, *a, **k: self.clone()  # noqa: E731
    for i, ln in enumerate((False, True)):
        torch.manual_seed(400 + i)
        m = RecurrentRGCN("convtranse", "uvrgcn", V, R, 0, 0, d, "sub", T, num_bases=100, num_basis=100,
                          num_hidden_layers=2, dropout=0.0, self_loop=True, skip_connect=False, layer_norm=ln,
                          input_dropout=0.0, hidden_dropout=0.0, feat_dropout=0.0, entity_prediction=True,
                          relation_prediction=True, use_cuda=True, gpu="cpu")
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        m.train()
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.eval()
        m.zero_grad()
        le, lr, ls = m.get_loss(glist, batch.clone(), None, True)
        loss = tw * le + (1 - tw) * lr + ls
        loss.backward()
        out = {"meta": np.array([V, R, d, T]), "batch": snaps[T], "task_weight": np.array(tw),
               "losses": np.array([float(x) for x in (le, lr, ls, loss)])}
        for t in range(T):
            out["snap%d" % t] = snaps[t]
        for k, v in sd.items():
            out["sd_" + k] = v.numpy().copy()
        for k, p in m.named_parameters():
            if p.grad is not None:
                out["grad_" + k] = p.grad.numpy().copy()
        save("train_rrgcn_%s.npz" % ("ln" if ln else "noln"), **out)
    torch.Tensor.cuda = lambda self, *a, **k: self  # noqa: E731


def gen_rrgcn(large=False):
    """rrgcn_{noln,ln}: V 256, R 64, d 64; large: rrgcn_ln_d200 at ICEWS14s' relation count
    (R = 230) and the paper's d = 200, V 1500, 3000 triples per snapshot."""
    V, R, d, T = (1500, 230, 200, 3) if large else (256, 64, 64, 3)
    snaps = snapshot_series(31 if large else 30, V, R, T + 1, 3000 if large else 120)
    glist = [rutils.build_sub_graph(V, R, s, False, "cpu") for s in snaps[:T]]
    test = torch.from_numpy(snaps[T][:200] if large else snaps[T])
    for i, ln in enumerate((True,) if large else (False, True)):
        torch.manual_seed(200 + i)
        m = RecurrentRGCN("convtranse", "uvrgcn", V, R, 0, 0, d, "sub", T, num_bases=100,
                          num_basis=100, num_hidden_layers=2, dropout=0.2, self_loop=True,
                          skip_connect=False, layer_norm=ln, input_dropout=0.2, hidden_dropout=0.2,
                          feat_dropout=0.2, entity_prediction=True, relation_prediction=True,
                          use_cuda=False, gpu="cpu")
        m.eval()
        with torch.no_grad():
            embs, _, h0, _, _ = m.forward(glist, None, False)
            all_tr, score, score_rel = m.predict(glist, R, None, test.clone(), False)
        out = {"meta": np.array([V, R, d, T]), "test": test.numpy(), "all_triples": all_tr.numpy(),
               "score": score.numpy(), "score_rel": score_rel.numpy(), "h0": h0.numpy(),
               "embs": torch.stack(embs).numpy()}
        for t in range(T):
            out["snap%d" % t] = snaps[t]
        for k, v in m.state_dict().items():
            out["sd_" + k] = v.numpy().copy()
        save("rrgcn_%s%s.npz" % ("ln" if ln else "noln", "_d200" if large else ""), **out)


def gen_score():
    gen = torch.Generator().manual_seed(5)
    B, N, d = 64, 1000, 200
    q = ball_points(gen, B, d)
    e = ball_points(gen, N, d)
    # near-duplicate queries (cancellation stress) and a boundary query
    q[0] = e[17] + 1e-4 * torch.randn(d, generator=gen)
    q[1] = e[500]
    q[2] = q[2] / q[2].norm() * 9.99
    bias = torch.randn(N, generator=gen) * 0.1
    tgt = torch.randint(0, N, (B,), generator=gen)
    c_r = 0.002 + 0.008 * torch.rand(B, generator=gen)
    scale = torch.tensor(1.3)
    margin = torch.tensor(0.7)
    out = {"q": q.numpy(), "e": e.numpy(), "bias": bias.numpy(), "target": tgt.numpy(),
           "c_r": c_r.numpy(), "scale": scale.numpy(), "margin": margin.numpy()}
    with torch.no_grad():
        out["score_plain"] = hdec._chunked_hyperbolic_dist_score(q, e, None, C, 128, 256).numpy()
        out["score_bias"] = hdec._chunked_hyperbolic_dist_score(
            q, e, bias, C, 128, 256, score_scale=scale, score_margin=margin).numpy()
        out["score_crel"] = hdec._chunked_hyperbolic_dist_score(
            q, e, bias, C, 128, 256, score_scale=scale, score_margin=margin, query_curvature=c_r,
            use_hyperbolic_distance=True).numpy()
        out["score_dist"] = hdec._chunked_hyperbolic_dist_score(
            q, e, None, C, 128, 256, score_scale=scale, score_margin=margin,
            use_hyperbolic_distance=True).numpy()
        out["ce_bias"] = hdec._chunked_hyperbolic_ce_loss(
            q, e, tgt, C, 256, candidate_bias=bias, q_chunk_size=128, score_scale=scale,
            score_margin=margin).numpy()
        out["ce_crel"] = hdec._chunked_hyperbolic_ce_loss(
            q, e, tgt, C, 256, candidate_bias=bias, q_chunk_size=128, score_scale=scale,
            score_margin=margin, query_curvature=c_r, use_hyperbolic_distance=True).numpy()
    save("score.npz", **out)


def gen_rank():
    rng = np.random.default_rng(6)
    V, R, B = 120, 10, 80
    snap = zipf_triples(rng, V, R, B, alpha=0.8)
    snap[40:50] = snap[0:10]
    snap[50:55, 2] = (snap[50:55, 2] + 1) % V  # same (s, r), another object
    snap[50:55, :2] = snap[0:5, :2]
    tr = torch.from_numpy(snap)
    inv = tr[:, [2, 1, 0]].clone()
    inv[:, 1] += R
    all_tr = torch.cat([tr, inv])
    score = torch.from_numpy(rng.standard_normal((2 * B, V)).astype(np.float32))
    score_rel = torch.from_numpy(rng.standard_normal((2 * B, 2 * R)).astype(np.float32))
    data = np.concatenate([snap, np.zeros((B, 1), np.int64)], 1)
    ans_e = rutils.load_all_answers_for_time_filter(data, R, V, False)[0]
    ans_r = rutils.load_all_answers_for_time_filter(data, R, V, True)[0]
    mrr_f, mrr, rank, frank = rutils.get_total_rank(all_tr, score.clone(), ans_e, 1000, 0)
    mrr_fr, mrr_r, rank_r, frank_r = rutils.get_total_rank(all_tr, score_rel.clone(), ans_r, 1000, 1)
    save("rank.npz", snap=snap, all_triples=all_tr.numpy(), score=score.numpy(),
         score_rel=score_rel.numpy(), rank=rank.numpy(), frank=frank.numpy(),
         rank_r=rank_r.numpy(), frank_r=frank_r.numpy(),
         mrr=np.array([mrr, mrr_f, mrr_r, mrr_fr]), meta=np.array([V, R]))


def gen_dataset():
    """A tiny dataset directory in the reference's on-disk format (knowledge_graph.py:189-206,
    :526-555) and what the reference's load_from_local + split_by_time (rgcn/utils.py:306-339)
    make of it.  entity2id.txt repeats one id under two names (num_nodes = len of the dict
    keyed by id, not the line count); the time column starts at a nonzero t and holds a
    one-triple snapshot."""
    from rgcn import knowledge_graph as kg
    root = os.path.join(OUT, "tkg_tiny")
    os.makedirs(root, exist_ok=True)
    rng = np.random.default_rng(7)
    V, R = 40, 6
    names = ["ent_%d" % i for i in range(V)] + ["ent_alias_7"]
    ids = list(range(V)) + [7]
    with open(os.path.join(root, "entity2id.txt"), "w") as f:
        f.writelines("%s\t%d\n" % (n, i) for n, i in zip(names, ids))
    with open(os.path.join(root, "relation2id.txt"), "w") as f:
        f.writelines("rel_%d\t%d\n" % (i, i) for i in range(R))
    t0 = 3
    splits = {"train": (0, 6), "valid": (6, 8), "test": (8, 10)}
    for name, (a, b) in splits.items():
        rows = []
        for t in range(a, b):
            n = 1 if t == 4 else int(rng.integers(5, 15))
            tr = np.stack([rng.integers(0, V, n), rng.integers(0, R, n), rng.integers(0, V, n)], 1)
            rows += [(int(x[0]), int(x[1]), int(x[2]), t0 + 24 * t) for x in tr]
        with open(os.path.join(root, name + ".txt"), "w") as f:
            f.writelines("%d\t%d\t%d\t%d\t0\n" % r for r in rows)
    data = kg.load_from_local(OUT, "tkg_tiny")
    out = {"num_nodes": np.array(data.num_nodes), "num_rels": np.array(data.num_rels)}
    for name in splits:
        arr = getattr(data, name)
        snaps = rutils.split_by_time(arr)
        out[name] = arr
        out[name + "_snap_len"] = np.array([len(x) for x in snaps])
        out[name + "_snaps"] = np.concatenate(snaps)
    save("dataset_tiny.npz", **out)


ANALYSIS_CASES = [
    ("uvrgcn_roth_beta", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False,
                              radius_anchor_beta=0.5)),
    ("lgcn_roth_ln", dict(encoder_name="lgcn", decoder_name="roth", layer_norm=True)),
    ("uvrgcn_murp_nores", dict(encoder_name="hyperbolic_uvrgcn", decoder_name="murp", layer_norm=False,
                               use_residual_evolution=False)),
]
SUMMARY_KEYS = ("curvature", "radius_delta_mean", "radius_delta_std", "dynamic_radius_mean", "static_radius_mean",
                "base_radius_mean", "anchor_beta", "avg_time_gate")
EVO_KEYS = ("delta_mean", "delta_std", "dynamic_radius_mean", "static_radius_mean", "base_radius_mean",
            "anchor_beta")
EMB_KEYS = ("mean_norm", "max_norm", "min_norm", "std_norm", "max_allowed", "pct_near_boundary")


def gen_analysis():
    """--run-analysis (analysis=True): the eval forward's gate_list and time-gate means, the
    radius-evolution stats, the predict embeddings' stats (log_embedding_stats, captured), then
    one training mini-batch (dropout 0): the init embeddings' stats, the loss components, the
    total gradient norm of log_gradient_stats and get_training_summary."""
    from hyperbolic_src import hyperbolic_model as hm
    V, R, T, d, tw = 256, 64, 3, 64, 0.7
    snaps = snapshot_series(60, V, R, T + 1, 120)
    rng = np.random.default_rng(61)
    radius_target = rng.uniform(0.5, 3.0, size=V).astype(np.float32)
    glist = [rutils.build_sub_graph(V, R, s, False, "cpu") for s in snaps[:T]]
    batch = torch.from_numpy(snaps[T])
    logged = {}
    orig = HyperbolicOps.log_embedding_stats

    def capture(x, name="embeddings", c=0.01):
        logged[name] = orig(x, name, c)
        return logged[name]

    for i, (tag, kw) in enumerate(ANALYSIS_CASES):
        torch.manual_seed(600 + i)
        base = dict(num_ents=V, num_rels=R, num_static_rels=0, num_words=0, h_dim=d, opn="sub",
                    sequence_len=T, num_bases=d // 2, num_hidden_layers=2, dropout=0.0, c=C,
                    self_loop=True, skip_connect=False, input_dropout=0.0, hidden_dropout=0.0,
                    feat_dropout=0.0, entity_prediction=True, relation_prediction=True,
                    use_cuda=False, gpu="cpu", radius_target=radius_target, radius_msg_gamma=0.15,
                    analysis=True)
        base.update(kw)
        m = HyperbolicRecurrentRGCN(**base)
        with torch.no_grad():
            for mod in (m.decoder_ob, m.rdecoder):
                if hasattr(mod, "score_margin"):
                    mod.score_margin.fill_(0.7)
                    mod.score_scale_raw.fill_(0.4)
            m.radius_static.add_(torch.randn(V) * 0.2)
            m.time_gate_bias.normal_(0, 0.5)  # gates away from one value
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        out = {"meta": np.array([V, R, d, T]), "batch": snaps[T], "radius_target": radius_target,
               "task_weight": np.array(tw)}
        for t in range(T):
            out["snap%d" % t] = snaps[t]
        for k, v in sd.items():
            out["sd_" + k] = v.numpy().copy()
        logged.clear()
        hm.HyperbolicOps.log_embedding_stats = staticmethod(capture)
        try:
            m.eval()
            with torch.no_grad():
                _, _, _, gate_list, degree_list = m.forward(glist, None, False)
                out["eval_gates"] = torch.stack(gate_list).numpy()
                out["eval_time_gate_values"] = np.array(m.training_stats["time_gate_values"])
                ev = m.temporal_radius_evolution.get_evolution_stats()
                out["eval_evolution"] = np.array([ev[k] for k in EVO_KEYS] if ev else [])
                m.predict(glist, R, None, batch.clone(), False)
            out["predict_emb_stats"] = np.array([logged["predict_embeddings"][k] for k in EMB_KEYS])
            m.train()
            for mod in m.modules():
                if isinstance(mod, torch.nn.BatchNorm1d):
                    mod.eval()
            m.zero_grad()
            le, lr, ls, lrad = m.get_loss(glist, batch.clone(), None, False)
            (tw * le + (1 - tw) * lr + ls + lrad).backward()
            out["init_emb_stats"] = np.array([logged["init_embeddings"][k] for k in EMB_KEYS])
        finally:
            hm.HyperbolicOps.log_embedding_stats = staticmethod(orig)
        lc = m.training_stats["loss_components"][-1]
        out["loss_components"] = np.array([lc[k] for k in ("loss_ent", "loss_rel", "loss_static", "loss_radius")])
        out["grad_norm"] = np.array(m.log_gradient_stats())
        out["train_time_gate_values"] = np.array(m.training_stats["time_gate_values"])
        summ = m.get_training_summary()
        out["summary_keys"] = np.array([k for k in SUMMARY_KEYS if k in summ])
        out["summary"] = np.array([float(summ[k]) for k in SUMMARY_KEYS if k in summ])
        assert set(summ) <= set(SUMMARY_KEYS), summ
        save("analysis_%s.npz" % tag, **out)


def gen_multistep():
    """get_total_rank filters `score` in place; --multi-step builds the next history
    snapshot from those filtered scores (hyperbolic_main.py:116-149)."""
    z = np.load(os.path.join(OUT, "rank.npz"))
    V, R = (int(v) for v in z["meta"])
    snap = z["snap"]
    all_tr = torch.from_numpy(z["all_triples"])
    data = np.concatenate([snap, np.zeros((len(snap), 1), np.int64)], 1)
    ans_e = rutils.load_all_answers_for_time_filter(data, R, V, False)[0]
    ans_r = rutils.load_all_answers_for_time_filter(data, R, V, True)[0]
    # ties at the top would leave torch.sort's order unspecified: shift the scores so the
    # filtered entries (-1e7) are the only ties, far below every top-k
    score = torch.from_numpy(z["score"]).clone()
    score_rel = torch.from_numpy(z["score_rel"]).clone()
    rutils.get_total_rank(all_tr, score, ans_e, 1000, 0)
    rutils.get_total_rank(all_tr, score_rel, ans_r, 1000, 1)
    k = 4
    snap_e = rutils.construct_snap(all_tr, V, R, score, k)
    snap_r = rutils.construct_snap_r(all_tr, V, R, score_rel, k)
    save("multistep.npz", filtered_score=score.numpy(), filtered_score_rel=score_rel.numpy(),
         snap_e=snap_e, snap_r=snap_r, topk=np.array([k]))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:] or ["graph", "ops", "union", "euclid", "lorentz", "models", "rrgcn",
                             "score", "rank", "train"]
    table = {"graph": gen_graph_indexing, "ops": gen_ops, "union": gen_layer_union,
             "euclid": gen_layer_euclid, "lorentz": gen_layer_lorentz, "models": gen_models,
             "rrgcn": gen_rrgcn, "rrgcn_large": lambda: gen_rrgcn(True), "score": gen_score, "rank": gen_rank, "train": gen_train,
             "models_large": gen_models_large, "dataset": gen_dataset, "train_curvature": gen_train_curvature,
             "multistep": gen_multistep, "analysis": gen_analysis}
    for w in which:
        table[w]()
