"""The config-5 decoder against the float64 oracle (-m gpu): BASELINE.json configs[4]'s scoring
shape, B = 1,024 RotH queries (512 test triples and their inverses) x all N = 1,000,000
entities, d = 200 (2 B N d = 410 GFLOP, the MFMA-bound launch).

The entity rows are Poincare rows shaped like a predict's output (exp0 of N(0, 1) rows at radii
U[0.5, 3.0], c = 0.01); decoder weights are bench.build_model's random init.  Checked:
  * the fused query front (regcn_roth_queries_f32) against oracle.model.entity_decoder's query
    sequence in float64 (hyperbolic_decoder.py:1065-1085) on all 1,024 queries;
  * k_score_f32_jobs (regcn_hyp_score_jobs_f32, the predict's scorer) on 64 query rows x all
    1M candidates against the proxy score of hyperbolic_decoder.py:89-179 (oracle.model.dist_score)
    in float64, chunked over the candidates: |delta| <= 1e-4 * max(1, |ref|);
  * the fused cross entropy (regcn_hyp_ce_f32, no B x N logits) of the same 64 queries against
    the float64 log-sum-exp over all 1M candidates minus the target logit (:182-307);
  * the candidate-sharded ranks (parallel.CandidateShard.range_ranks over the 8 ranks' owner
    ranges of an 8-GPU owner layout, counts summed as their all_reduce sums them) equal the
    ranks counted from the full score matrix, bit for bit, for all 1,024 queries."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
C = 0.01


def test_config5_decoder_vs_float64():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bench
    from oracle import model as OM
    from oracle import ops
    from regcn_amd.hyperbolic_decoder import roth_pair_queries, roth_pair_scores
    from regcn_amd.parallel import CandidateShard, OwnerLayout
    from regcn_amd.synthetic import CONFIGS
    cfg = CONFIGS["synthetic_1m"]
    V, R, d = cfg["V"], cfg["R"], 200
    model = bench.build_model(cfg, d, DEV, seed=11)
    dec, rdec = model.decoder_ob, model.rdecoder
    gen = torch.Generator(device=DEV).manual_seed(3)
    with torch.no_grad():
        emb = ops.apply_radius(ops.exp0(torch.randn(V, d, device=DEV, generator=gen), C),
                               torch.rand(V, device=DEV, generator=gen) * 2.5 + 0.5, C).contiguous()
        rel = (torch.randn(2 * R, d, device=DEV, generator=gen) * 0.3).contiguous()
        rng = np.random.default_rng(4)
        test = torch.from_numpy(np.stack([rng.integers(0, V, 512), rng.integers(0, R, 512),
                                          rng.integers(0, V, 512)], 1)).to(DEV)
        all_tr, q_ent, q_rel, cand = roth_pair_queries(dec, rdec, emb, rel, test, R)
        score, _ = roth_pair_scores(dec, rdec, emb, q_ent, q_rel, cand)
        B = q_ent.shape[0]
        assert B == 1024 and score.shape == (B, V)
        sd = {k: v.detach().double() for k, v in model.state_dict().items()}
        e64, r64 = emb.double(), rel.double()
        # the query front vs the reference sequence in float64
        p = "decoder_ob."
        s_idx, r_idx = all_tr[:, 0].long(), all_tr[:, 1].long()
        s_tan = ops.log0(ops.project(e64[s_idx], C), C)
        s_tan = s_tan + OM._lin(sd, p + "reshape_fc2", torch.relu(OM._lin(sd, p + "reshape_fc1", s_tan)))
        rr = r64[r_idx]
        q0 = ops.exp0(OM.givens_rotation(s_tan, OM._lin(sd, p + "rot_proj", rr)), C)
        t_r = ops.project(ops.exp0(OM._lin(sd, p + "trans_proj", rr), C), C)
        q_ref = ops.mobius_add(ops.project(q0, C), t_r, C)
        err_q = float(((q_ent.double() - q_ref).abs() / q_ref.abs().clamp_min(1.0)).max())
        assert err_q <= 1e-4, err_q
        # 64 query rows x all 1M candidates in float64, chunked over the candidates
        pick = torch.arange(0, B, B // 64, device=DEV)
        q64 = q_ent[pick].double()
        scale = OM._scale(sd, p)
        margin = sd[p + "score_margin"]
        tgt = all_tr[pick, 2].long()
        worst = 0.0
        m_run = torch.full((64,), -float("inf"), device=DEV, dtype=torch.float64)
        s_run = torch.zeros(64, device=DEV, dtype=torch.float64)
        t_logit = torch.zeros(64, device=DEV, dtype=torch.float64)
        step = 8192
        for a in range(0, V, step):
            b = min(V, a + step)
            ref = OM.dist_score(q64, e64[a:b], None, C, scale, margin, chunk=16)
            got = score[pick, a:b].double()
            worst = max(worst, float(((got - ref).abs() / ref.abs().clamp_min(1.0)).max()))
            mx = torch.maximum(m_run, ref.max(1).values)
            s_run = s_run * torch.exp(m_run - mx) + torch.exp(ref - mx[:, None]).sum(1)
            m_run = mx
            inside = (tgt >= a) & (tgt < b)
            if bool(inside.any()):
                rows = torch.nonzero(inside).flatten()
                t_logit[rows] = ref[rows, tgt[rows] - a]
        assert worst <= 1e-4, "k_score_f32_jobs vs float64: %.3g" % worst
        loss_ref = m_run + torch.log(s_run) - t_logit
        loss = dec.loss(emb, rel, all_tr, reduction="none")[pick].double()
        err_ce = float(((loss - loss_ref).abs() / loss_ref.abs().clamp_min(1.0)).max())
        assert err_ce <= 1e-4, "fused CE vs float64: %.3g" % err_ce
        # candidate-sharded ranks (8 owner ranges) == ranks counted on the full scores
        ts = score.gather(1, all_tr[:, 2:3].long())
        full_rank = (score > ts).sum(1) + 1
        lay = OwnerLayout(V, 8, 4)
        kw = dict(scale=dec.score_scale_raw, margin=dec.score_margin, raw_scale=True)
        ts0 = CandidateShard(V, 0, 8, None).target_scores(q_ent, emb, None, all_tr[:, 2], dec.c, **kw)
        assert torch.equal(ts0, ts.flatten()), "target scores differ from the full scoring's bits"
        tot = torch.zeros(B, device=DEV, dtype=torch.long)
        for k in range(8):
            sh = CandidateShard(V, k, 8, None, ranges=lay.ranges(k))
            raw, _ = sh.range_ranks(q_ent, emb, None, dec.c, ts0, **kw)
            tot += raw - 1
        assert torch.equal(tot + 1, full_rank)
    print("config-5 decoder: query err %.2e, score err %.2e (64 x 1M), CE err %.2e" % (err_q, worst, err_ce))
