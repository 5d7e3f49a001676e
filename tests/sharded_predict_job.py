"""One rank of the sharded-predict GPU test (tests/test_gpu_sharded.py), launched by
torch.distributed.run: the snapshots of a dataset-shaped golden partitioned over the ranks
(owner and edge partitions), HyperbolicRecurrentRGCN.forward and predict_ranks (candidate-
sharded entity ranks) against the same model run unsharded in this process.  Rank 0 writes
a JSON summary to argv[1]."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "re-gcn_amd"))


def main(out_path, tag):
    from gpu_helpers import build_hyperbolic_model
    from regcn_amd import ranking
    from regcn_amd.parallel import ShardedGraph, complete
    dist.init_process_group(os.environ.get("REGCN_DIST_BACKEND", "gloo"))
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    z = np.load(os.path.join(HERE, "golden", "model_%s.npz" % tag))
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, dev)
    test = torch.from_numpy(z["test"]).to(dev)
    ans = ranking.load_all_answers_for_filter(z["test"], R, False)
    ans_r = ranking.load_all_answers_for_filter(z["test"], R, True)
    res = {"world": world, "tag": tag}
    with torch.no_grad():
        embs, _, h0, _, _ = m.forward(glist, None, True)
        ref_emb = embs[-1].clone()
        _, (re_, fe_), (rr_, fr_) = m.predict_ranks(glist, R, None, test, True, ans, ans_r)
        for part in ("owner", "edge"):
            for chunks in ((1, 3) if part == "owner" else (1,)):
                sg = [ShardedGraph(g, part, chunks=chunks) for g in glist]
                # forward itself completes the last state (the owner partition's other rows)
                e2, _, h02, _, _ = m.forward(sg, None, True)
                _, (re2, fe2), (rr2, fr2) = m.predict_ranks(sg, R, None, test, True, ans, ans_r)
                # the candidate-sharded decoder alone, on the unsharded encoder outputs: the
                # same ranks bit for bit (the partitions sum rows in another order, so the
                # end-to-end ranks may differ at near ties only)
                m.forward = lambda g_list, s, u: (embs, None, h0, [], [])
                _, (re3, fe3), (rr3, fr3) = m.predict_ranks(sg, R, None, test, True, ans, ans_r)
                del m.forward
                d_e = (re2.cpu() - re_.cpu()).abs()
                key = "%s_%d" % (part, chunks)
                res[key] = {
                    "emb_err": float(((e2[-1] - ref_emb).abs() / ref_emb.abs().clamp_min(1.0)).max()),
                    "h0_err": float((h02 - h0).abs().max()),
                    "dec_ent_rank_equal": bool(torch.equal(re3.cpu(), re_.cpu()) and torch.equal(fe3.cpu(), fe_.cpu())),
                    "dec_rel_rank_equal": bool(torch.equal(rr3.cpu(), rr_.cpu()) and torch.equal(fr3.cpu(), fr_.cpu())),
                    "ent_rank_queries_differing": int((d_e > 0).sum()), "queries": int(d_e.numel()),
                    "ent_rank_max_diff": int(d_e.max()),
                }
        # --run-analysis under the owner partition: the non-fused timestep reads every row of
        # the cell output, which the sharded forward completes first
        m.run_analysis = True
        try:
            ea, _, _, ga, _ = m.forward(glist, None, True)
            ref_a = ea[-1].clone()
            ref_g = [g.clone() for g in ga]
            sg = [ShardedGraph(g, "owner", chunks=2) for g in glist]
            eb, _, _, gb, _ = m.forward(sg, None, True)
            hist = [complete(e) for e in eb]
            res["owner_analysis"] = {
                "emb_err": float(((eb[-1] - ref_a).abs() / ref_a.abs().clamp_min(1.0)).max()),
                "hist_err": float(max(((a - b).abs() / b.abs().clamp_min(1.0)).max() for a, b in zip(hist, ea))),
                "gate_err": float(max((a - b).abs().max() for a, b in zip(gb, ref_g))) if ref_g else 0.0,
            }
        finally:
            m.run_analysis = False
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "uvrgcn_roth_r512_d200")
