"""--run-analysis on the HIP path (hyperbolic_main.py:716; the verdict's row N1) against the
reference's own analysis=True run (tests/golden/analysis_*.npz, tools/goldens/make_golden.py
analysis):
  * eval forward: gate_list (each timestep's time gate, V x d, hyperbolic_model.py:852-856) and
    training_stats["time_gate_values"], from the analysis variant of the timestep kernel
    (regcn_timestep_analysis_f32); TemporalRadiusEvolution.get_evolution_stats()
    (hyperbolic_ops.py:426-434); the predict embeddings' norm stats (:932-933);
  * one training mini-batch: the init embeddings' stats (:791-792), the loss components
    (:1076-1082), log_gradient_stats' total norm (:1090-1108) and get_training_summary
    (:1110-1127).
Tolerance 1e-4 * max(1, |ref|); the gradient norm 2e-3 relative (the training
tests' bound on the reference's own fp32 gradients)."""
import numpy as np
import pytest
import torch

from gpu_helpers import assert_close
from regcn_amd import graph as G

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
C = 0.01
CASES = {
    "uvrgcn_roth_beta": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="roth", layer_norm=False,
                             radius_anchor_beta=0.5),
    "lgcn_roth_ln": dict(encoder_name="lgcn", decoder_name="roth", layer_norm=True),
    "uvrgcn_murp_nores": dict(encoder_name="hyperbolic_uvrgcn", decoder_name="murp", layer_norm=False,
                              use_residual_evolution=False),
}
EVO = ("delta_mean", "delta_std", "dynamic_radius_mean", "static_radius_mean", "base_radius_mean", "anchor_beta")
EMB = ("mean_norm", "max_norm", "min_norm", "std_norm", "max_allowed", "pct_near_boundary")


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
              radius_msg_gamma=0.15, analysis=True)
    kw.update(CASES[tag])
    m = HyperbolicRecurrentRGCN(**kw)
    m.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd_")}, strict=True)
    glist = [G.build_sub_graph(V, R, z["snap%d" % t], True, DEV) for t in range(T)]
    return m.to(DEV), glist


@pytest.mark.parametrize("tag", list(CASES))
def test_analysis_vs_reference(golden, tag):
    z = golden("analysis_%s.npz" % tag)
    m, glist = build(z, tag)
    V, R, d, T = (int(v) for v in z["meta"])
    batch = torch.from_numpy(z["batch"]).to(DEV)
    m.eval()
    with torch.no_grad():
        _, _, _, gate_list, degree_list = m.forward(glist, None, True)
        assert len(gate_list) == T and degree_list == []
        assert_close(torch.stack(gate_list), z["eval_gates"], what="gate_list")
        assert_close(m.training_stats["time_gate_values"], z["eval_time_gate_values"], what="time_gate_values")
        ev = m.temporal_radius_evolution.get_evolution_stats()
        if z["eval_evolution"].size:
            assert_close([ev[k] for k in EVO], z["eval_evolution"], what="evolution stats")
        else:
            assert ev is None
        m.predict(glist, R, None, batch.clone(), True)
    from regcn_amd.analysis import embedding_dict
    s = embedding_dict(m.embedding_stats["predict_embeddings"], "predict_embeddings", C)
    assert_close([s[k] for k in EMB], z["predict_emb_stats"], what="predict embedding stats")
    m.train()
    m.zero_grad()
    tw = float(z["task_weight"])
    le, lr, ls, lrad = m.get_loss(glist, batch, None, True)
    (tw * le + (1 - tw) * lr + ls.sum() + lrad).backward()
    s = embedding_dict(m.embedding_stats["init_embeddings"], "init_embeddings", C)
    assert_close([s[k] for k in EMB], z["init_emb_stats"], what="init embedding stats")
    lc = m.training_stats["loss_components"][-1]
    assert_close([lc[k] for k in ("loss_ent", "loss_rel", "loss_static", "loss_radius")], z["loss_components"],
                 what="loss components")
    gn = m.log_gradient_stats()
    np.testing.assert_allclose(float(gn), float(z["grad_norm"]), rtol=2e-3)
    assert len(m.training_stats["gradient_norms"]) == 1
    summ = m.get_training_summary()
    assert list(summ) == [str(k) for k in z["summary_keys"]]
    assert_close([summ[str(k)] for k in z["summary_keys"]], z["summary"], what="training summary")


def test_analysis_forward_matches_plain(golden):
    """The analysis variant of the timestep kernel writes the same embeddings as the plain one."""
    z = golden("analysis_uvrgcn_roth_beta.npz")
    m, glist = build(z, "uvrgcn_roth_beta")
    m.eval()
    with torch.no_grad():
        a = [e.clone() for e in m.forward(glist, None, True)[0]]
        m.run_analysis = False
        b = m.forward(glist, None, True)[0]
    for x, y in zip(a, b):
        assert_close(x, y, 1e-5, "analysis vs fused forward")
