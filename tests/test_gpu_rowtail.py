"""The large-snapshot layer path (regcn_layer_rowtail_f32, csrc/rowtail.hip: the inline
in-edge rows gathered into the agg buffer, then the 64-row MFMA tail with in-wave row
reductions and the time gate computed by the cell's first layer) against the reference.

The path is taken by snapshots of >= hyperbolic_layers.ROWTAIL_MIN_ROWS rows (config 5); here
the threshold is lowered so the d = 200 reference-run model goldens (tests/golden/model_*_d200:
hub rows over the inline budget, R2 = 512, |E| = 80k, history 7, the Lorentz encoder with layer
norm) run through it: history embeddings, relation state and both decoders' scores within
1e-4 * max(1, |ref|).  Also a direct comparison with the fused 16-row kernel
on a 70k-row snapshot (Zipf hubs, rows without in-edges), union / Lorentz / euclid, with and
without the timestep, and with the timestep's gate computed in-kernel."""
import numpy as np
import pytest
import torch

from gpu_helpers import assert_close, build_hyperbolic_model

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
C = 0.01


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.fixture
def rowtail_everywhere(monkeypatch):
    from regcn_amd import hyperbolic_layers as HL
    monkeypatch.setattr(HL, "ROWTAIL_MIN_ROWS", 1)
    return HL


@pytest.mark.parametrize("tag", ["uvrgcn_roth_r512_d200", "uvrgcn_roth_e80k_d200", "uvrgcn_roth_h7_d200",
                                 "lgcn_roth_h7_d200"])
def test_rowtail_model_vs_golden(golden, rowtail_everywhere, tag):
    from regcn_amd import _lib
    z = golden("model_%s.npz" % tag)
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, DEV)
    m.use_phases = False  # the per-layer launches (the phases are the dataset-size schedule)
    calls = []
    _lib.EVENT_TRACE = calls
    try:
        with torch.no_grad():
            embs, _, h0, _, _ = m.forward(glist, None, True)
            all_tr, score, score_rel = m.predict(glist, R, None, torch.from_numpy(z["test"]).to(DEV), True)
    finally:
        _lib.EVENT_TRACE = None
    names = {n for n, _ in calls}
    assert "regcn_layer_rowtail_f32(step)" in names and "regcn_layer_f32(step)" not in names, names
    assert_close(embs[-1], z["embs_last"], what="last history embedding")
    assert_close(h0, z["h0"], what="h_0")
    assert_close(score, z["score"], what="entity score")
    assert_close(score_rel, z["score_rel"], what="relation score")


def _zipf_snapshot(V, R, n, seed):
    from regcn_amd.synthetic import zipf_triples
    rng = np.random.default_rng(seed)
    return zipf_triples(rng, V, R, n)


@pytest.mark.parametrize("encoder,residual,ln,d", [("hyperbolic_uvrgcn", True, False, 200), ("lgcn", True, True, 200),
                                                   ("hyperbolic_uvrgcn", False, True, 200),
                                                   # column-tile buckets wider than ceil(d / 16): NT = 8 at d = 96 /
                                                   # 100, NT = 4 at d = 32 (the tiles past d must not be stored)
                                                   ("hyperbolic_uvrgcn", True, False, 96),
                                                   ("hyperbolic_uvrgcn", True, True, 100), ("lgcn", True, False, 32)])
def test_rowtail_matches_fused_layers(encoder, residual, ln, d):
    """A 70k-row snapshot window (> ROWTAIL_MIN_ROWS): the per-layer forward with the 64-row
    tail equals the fused 16-row kernel's within 1e-4 * max(1, |ref|) (the products sum in
    another k order), and so does the step layer computing its own time gate.  The widths
    below 200 run the tail with more column tiles than d fills (csrc/rowtail.hip launch_tail's
    NT buckets): a store past column d would land in the next row."""
    from regcn_amd import graph as G
    from regcn_amd import hyperbolic_layers as HL
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    V, R, T = 70_000, 64, 2
    torch.manual_seed(7)
    m = HyperbolicRecurrentRGCN("roth", encoder, V, R, 0, 0, d, "sub", T, num_bases=d // 2, num_hidden_layers=2,
                                dropout=0.0, c=C, self_loop=True, layer_norm=ln, entity_prediction=True,
                                relation_prediction=True, use_cuda=True, gpu=0, use_residual_evolution=residual,
                                radius_msg_gamma=0.15).to(DEV).eval()
    m.use_phases = False
    glist = [G.build_sub_graph(V, R, _zipf_snapshot(V, R, 400_000, 30 + t), True, DEV) for t in range(T)]
    assert all(g.n_heavy > 0 and g.n_pos < V for g in glist)
    with torch.no_grad():
        old = HL.ROWTAIL_MIN_ROWS
        try:
            HL.ROWTAIL_MIN_ROWS = 0
            ref = [e.clone() for e in m.forward(glist, None, True)[0]]
            HL.ROWTAIL_MIN_ROWS = 1
            got = m.forward(glist, None, True)[0]
            for a, b in zip(got, ref):
                assert_close(a, b, what="rowtail vs fused")
            # the step layer's in-kernel gate (the first layer computes no gate rows)
            layer0 = m.rgcn.layers[0]
            real = layer0.forward
            layer0.forward = lambda *a, **k: real(*a, **{**k, "gate": None})
            try:
                got2 = m.forward(glist, None, True)[0]
            finally:
                del layer0.forward
            for a, b in zip(got2, ref):
                assert_close(a, b, what="rowtail (in-kernel gate) vs fused")
        finally:
            HL.ROWTAIL_MIN_ROWS = old


def test_predict_last_step_writes_h_only(golden, rowtail_everywhere, monkeypatch):
    """predict's last timestep on the 64-row tail writes h only (StepSpec.need_xr: its x and |h|
    are read by nothing): the scores are bit for bit those of the run that writes them, and the
    last state carries no tangent cache (a later tangent_of recomputes it instead of reading
    unwritten rows)."""
    from regcn_amd import hyperbolic_model as HM
    z = golden("model_uvrgcn_roth_r512_d200.npz")
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, "uvrgcn_roth_r512_d200", DEV)
    m.use_phases = False
    test = torch.from_numpy(z["test"]).to(DEV)
    outs = {}
    for skip in (False, True):
        monkeypatch.setattr(HM, "LAST_SKIP_XR", skip)
        with torch.no_grad():
            outs[skip] = [t.clone() for t in m.predict(glist, R, None, test, True)[1:]]
            last = m._forward_last_h(glist, None, True)[0][-1]
        assert (getattr(last, "_regcn_xr", None) is None) == skip, "tangent cache on the last state"
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)
    assert_close(outs[True][0], z["score"], what="entity score")
