"""`hyperbolic_main.py` command line on the HIP path (mirror of hyperbolic_src/hyperbolic_main.py
:709-843, evaluation branch :60-161).

    python -m regcn_amd.cli -d ICEWS14s --test --encoder lgcn --decoder roth --gpu 0 \
        --data-dir ../data --checkpoint ../models/<name>

Every reference flag is accepted with the reference default.  Datasets use the reference's
on-disk format (`<data-dir>/<dataset>/{train,valid,test}.txt` rows `s\\tr\\to\\tt`,
`entity2id.txt` / `relation2id.txt` `name\\tid`, opened read-only);
`-d synthetic:<config>` evaluates a generated snapshot series of a
`regcn_amd.synthetic.CONFIGS` shape instead.  Checkpoints are read with
`torch.load(weights_only=True)` (`{'state_dict': ..., 'epoch': ...}` as the reference saves
them); without one the model keeps its random initialisation.

Without `--test` the model trains (hyperbolic_main.py:505-705): epochs over the shuffled
training snapshots, each one's history window as input, its triples in `--triple-batch-size`
mini-batches whose gradients accumulate, gradient clipping and one Adam step per snapshot,
validation every `--evaluate-every` epochs saving the best raw MRR to the checkpoint, early
stop after 20 epochs without improvement, then the test set on the best checkpoint.  The
forward and backward run on the HIP kernels (training.py / autograd.py); snapshot graphs
are built once on the device and reused across epochs (the reference rebuilds them per
sample, :560).  Out-of-scope features (static graph, EST, fhnn/hgat, Riemannian Adam) raise.
"""
import argparse
import contextlib
import logging
import os
import random
import sys
import time

import numpy as np
import torch

from . import ranking
from .graph import build_sub_graph
from .training import GraphedSteps
from .weights import bump_versions, invalidate

logger = logging.getLogger("regcn_amd.cli")


def build_parser():
    p = argparse.ArgumentParser(description="Hyperbolic Temporal RE-GCN (MI355X HIP path)")
    a = p.add_argument
    a("--gpu", type=int, default=-1)
    a("--batch-size", type=int, default=1)
    a("-d", "--dataset", type=str, required=True)
    a("--test", action="store_true", default=False)
    a("--run-analysis", action="store_true", default=False)
    a("--multi-step", action="store_true", default=False)
    a("--topk", type=int, default=10)
    a("--add-static-graph", action="store_true", default=False)
    a("--relation-evaluation", action="store_true", default=False)
    a("--curvature", type=float, default=0.01)
    a("--learn-curvature", action="store_true", default=False)
    a("--curvature-min", type=float, default=1e-4)
    a("--curvature-max", type=float, default=1e-1)
    a("--curvature-warmup-epochs", type=int, default=0)
    a("--disable-residual", action="store_true", default=False)
    a("--radius-alpha", type=float, default=0.5)
    a("--radius-beta", type=float, default=0.5)
    a("--radius-min", type=float, default=0.5)
    a("--radius-max", type=float, default=3.0)
    a("--radius-lambda", type=float, default=0.02)
    a("--radius-epsilon", type=float, default=0.1)
    a("--radius-anchor-beta", type=float, default=1.0)
    a("--radius-msg-gamma", type=float, default=0.15)
    a("--weight", type=float, default=1)
    a("--task-weight", type=float, default=0.7)
    a("--discount", type=float, default=1)
    a("--angle", type=int, default=10)
    a("--encoder", type=str, default="hyperbolic_uvrgcn", choices=["hyperbolic_uvrgcn", "fhnn", "lgcn", "hgat"])
    a("--attn-heads", type=int, default=4)
    a("--dropout", type=float, default=0.2)
    a("--skip-connect", action="store_true", default=False)
    a("--n-hidden", type=int, default=200)
    a("--opn", type=str, default="sub")
    a("--n-bases", type=int, default=100)
    a("--n-layers", type=int, default=2)
    a("--self-loop", action="store_true", dest="self_loop", default=True)
    a("--no-self-loop", action="store_false", dest="self_loop")
    a("--layer-norm", action="store_true", default=False)
    a("--relation-prediction", action="store_true", default=False)
    a("--entity-prediction", action="store_true", default=False)
    a("--n-epochs", type=int, default=500)
    a("--lr", type=float, default=0.001)
    a("--grad-norm", type=float, default=1.0)
    a("--evaluate-every", type=int, default=1)
    a("--triple-batch-size", type=int, default=64)
    a("--reuse-encoder", action=argparse.BooleanOptionalAction, default=True,
      help="one encoder forward per training snapshot for all its mini-batches (same gradients; "
           "--no-reuse-encoder recomputes it per mini-batch as hyperbolic_main.py does)")
    a("--hip-graph", action="store_true",
      help="replay each training sample's whole step (forward, backward, clip, Adam) from a HIP graph "
           "captured after its first step (single process; same math, dropout masks from the graph-safe "
           "generator)")
    a("--decoder", type=str, default="hyperbolic_convtranse", choices=["hyperbolic_convtranse", "murp", "roth", "atth"])
    a("--input-dropout", type=float, default=0.2)
    a("--hidden-dropout", type=float, default=0.2)
    a("--feat-dropout", type=float, default=0.2)
    a("--query-chunk-size", type=int, default=128)
    a("--candidate-chunk-size", type=int, default=256)
    a("--hyp-init-scale", type=float, default=1e-3)
    a("--hyp-score-scale-init", type=float, default=1.0)
    a("--hyp-score-margin-init", type=float, default=1.0)
    a("--plus-entity-euclidean-bias", action="store_true", default=False)
    a("--plus-relation-specific-curvature", action="store_true", default=False)
    a("--train-history-len", type=int, default=10)
    a("--test-history-len", type=int, default=20)
    a("--use-est", action="store_true", default=False)
    a("--est-history-len", type=int, default=32)
    a("--est-state-alpha", type=float, default=0.2)
    a("--est-encoder", type=str, default="gru")
    a("--use-time-aware-negative", action="store_true", default=False)
    a("--verbose", action="store_true", default=False)
    a("--log-file", action="store_true", default=False)
    a("--log-interval", type=int, default=1)
    a("--use-riemannian-adam", action="store_true", default=False)
    # build-only options
    a("--data-dir", type=str, default="../data", help="dataset root (reference: ../data)")
    a("--checkpoint", type=str, default=None, help="state checkpoint (torch.save of {'state_dict', 'epoch'})")
    a("--synthetic-snapshots", type=int, default=12, help="snapshots generated for -d synthetic:<config>")
    a("--seed", type=int, default=None, help="seed python/numpy/torch RNGs (snapshot shuffle, dropout, init)")
    a("--max-train-snapshots", type=int, default=None, help="train on at most this many snapshots per epoch")
    a("--shard", type=str, default="none", choices=["none", "owner", "edge"],
      help="--test with several ranks (torchrun): partition every snapshot over the ranks (destination "
           "owners + all-gather, or edge slices + all-reduce) and the entity candidates of the decoder "
           "(SURVEY.md §8(e)); default: rank 0 evaluates alone")
    return p


def _unsupported(args):
    bad = [("--add-static-graph", args.add_static_graph), ("--use-est", args.use_est),
           ("--use-time-aware-negative", args.use_time_aware_negative),
           ("--use-riemannian-adam", args.use_riemannian_adam),
           ("--encoder %s" % args.encoder, args.encoder in ("fhnn", "hgat"))]
    return [name for name, on in bad if on]


def load_dataset(args):
    """(num_nodes, num_rels, train, valid, test) with time in column 3 (reference
    knowledge_graph.load_from_local / _read_triplets_as_list)."""
    if args.dataset.startswith("synthetic:"):
        from .synthetic import CONFIGS, snapshot_series
        cfg = CONFIGS[args.dataset.split(":", 1)[1]]
        snaps = snapshot_series(0, cfg["V"], cfg["R"], args.synthetic_snapshots, cfg["per_snap"])
        rows = [np.concatenate([s, np.full((len(s), 1), t)], 1) for t, s in enumerate(snaps)]
        n = len(rows)
        tr, va = int(n * 0.7), int(n * 0.85)
        cat = lambda rs: np.concatenate(rs) if rs else np.zeros((0, 4), np.int64)  # noqa: E731
        return cfg["V"], cfg["R"], cat(rows[:tr]), cat(rows[tr:va]), cat(rows[va:])
    root = os.path.join(args.data_dir, args.dataset)

    def read(name):
        with open(os.path.join(root, name), "r") as f:  # reference opens 'r+' (fails read-only)
            return np.array([[int(v) for v in line.strip().split("\t")[:4]] for line in f if line.strip()],
                            dtype=np.int64).reshape(-1, 4)

    def count(name):
        """len of the {id: name} dict of knowledge_graph._read_dictionary (:526-532): ids
        repeated under several names count once."""
        with open(os.path.join(root, name), "r") as f:
            return len({int(line.strip().split("\t")[1]) for line in f if line.strip()})
    return count("entity2id.txt"), count("relation2id.txt"), read("train.txt"), read("valid.txt"), read("test.txt")


def radius_targets(snapshots, num_nodes, alpha=0.5, beta=0.5, radius_min=0.5, radius_max=3.0):
    """hyperbolic_main.py:164-185 (_compute_radius_targets)."""
    neigh = [set() for _ in range(num_nodes)]
    freq = np.zeros(num_nodes, dtype=np.float64)
    for snap in snapshots:
        if len(snap) == 0:
            continue
        freq += np.bincount(snap[:, 0], minlength=num_nodes)
        freq += np.bincount(snap[:, 2], minlength=num_nodes)
        for s, d in zip(snap[:, 0].tolist(), snap[:, 2].tolist()):
            neigh[s].add(d)
            neigh[d].add(s)
    deg = np.array([len(n) for n in neigh], dtype=np.float64)
    score = alpha * np.log1p(deg) + beta * np.log1p(freq)
    if score.max() - score.min() < 1e-9:
        normed = np.full_like(score, 0.5)
    else:
        normed = (score - score.min()) / (score.max() - score.min())
    return radius_min + (radius_max - radius_min) * normed


def build_model(args, num_nodes, num_rels, train_list, device):
    from .hyperbolic_model import HyperbolicRecurrentRGCN
    rt = radius_targets(train_list, num_nodes, args.radius_alpha, args.radius_beta, args.radius_min,
                        args.radius_max)
    m = HyperbolicRecurrentRGCN(
        decoder_name=args.decoder, encoder_name=args.encoder, num_ents=num_nodes, num_rels=num_rels,
        num_static_rels=0, num_words=0, h_dim=args.n_hidden, opn=args.opn, sequence_len=args.train_history_len,
        num_bases=args.n_bases, num_hidden_layers=args.n_layers, dropout=args.dropout, c=args.curvature,
        self_loop=args.self_loop, skip_connect=args.skip_connect, layer_norm=args.layer_norm,
        input_dropout=args.input_dropout, hidden_dropout=args.hidden_dropout, feat_dropout=args.feat_dropout,
        weight=args.weight, discount=args.discount, angle=args.angle, use_static=False,
        entity_prediction=args.entity_prediction, relation_prediction=args.relation_prediction,
        use_cuda=device.type == "cuda", gpu=args.gpu, analysis=args.run_analysis,
        learn_curvature=args.learn_curvature, use_residual_evolution=not args.disable_residual,
        radius_target=rt.astype(np.float32), radius_lambda=args.radius_lambda, radius_min=args.radius_min,
        radius_max=args.radius_max, radius_epsilon=args.radius_epsilon, radius_anchor_beta=args.radius_anchor_beta,
        curvature_min=args.curvature_min, curvature_max=args.curvature_max, num_heads=args.attn_heads,
        query_chunk_size=args.query_chunk_size, candidate_chunk_size=args.candidate_chunk_size,
        hyp_init_scale=args.hyp_init_scale, hyp_score_scale_init=args.hyp_score_scale_init,
        hyp_score_margin_init=args.hyp_score_margin_init,
        use_entity_euclidean_bias=args.plus_entity_euclidean_bias,
        use_relation_specific_curvature=args.plus_relation_specific_curvature,
        radius_msg_gamma=args.radius_msg_gamma)
    return m.to(device)


def test(model, history_list, test_list, num_rels, num_nodes, device, all_ans_list, all_ans_r_list, args):
    """hyperbolic_main.py:60-161: roll the history window over the test snapshots, predict,
    rank (raw + time-filtered; entity and relation), return the four MRRs."""
    ranks_raw, ranks_filter, ranks_raw_r, ranks_filter_r = [], [], [], []
    import torch.distributed as dist
    shard = getattr(args, "shard", "none") if dist.is_initialized() and dist.get_world_size() > 1 else "none"
    model.eval()
    input_list = [snap for snap in history_list[-args.test_history_len:]]
    graphs = {}
    # the pass is one batch of predicts: parameter-only states once (bit-identical results)
    share = getattr(model, "shared_parameter_states", None)
    with torch.no_grad(), share(args.test_history_len) if share else contextlib.nullcontext():
        for time_idx, test_snap in enumerate(test_list):
            glist = []
            for s in input_list:  # snapshot graphs cached by identity across the window
                key = id(s)
                if key not in graphs:
                    g = build_sub_graph(num_nodes, num_rels, s, True, device)
                    if shard != "none":
                        from .parallel import ShardedGraph
                        g = ShardedGraph(g, shard)
                    graphs[key] = (s, g)
                glist.append(graphs[key][1])
            tt = torch.from_numpy(np.asarray(test_snap, dtype=np.int64)).to(device)
            if shard != "none":  # partitioned snapshots and candidate-sharded entity ranks
                test_triples, (re_, fe), (rr, fr) = model.predict_ranks(
                    glist, num_rels, None, tt, True, all_ans_list[time_idx], all_ans_r_list[time_idx])
                score = score_r = None
            else:
                test_triples, score, score_r = model.predict(glist, num_rels, None, tt, True)
                _, _, rr, fr = ranking.get_total_rank(test_triples, score_r, all_ans_r_list[time_idx], 1000, 1)
                _, _, re_, fe = ranking.get_total_rank(test_triples, score, all_ans_list[time_idx], 1000, 0)
            ranks_raw_r.append(rr)
            ranks_filter_r.append(fr)
            ranks_raw.append(re_)
            ranks_filter.append(fe)
            if args.multi_step and score is None:
                raise SystemExit("--multi-step builds the next history from the full score matrix: not with --shard")
            if args.multi_step:
                pred = (ranking.construct_snap_r(test_triples, num_nodes, num_rels, score_r, args.topk)
                        if args.relation_evaluation else
                        ranking.construct_snap(test_triples, num_nodes, num_rels, score, args.topk))
                if len(pred):
                    input_list.pop(0)
                    input_list.append(pred)
            else:
                input_list.pop(0)
                input_list.append(test_snap)
            live = {id(s) for s in input_list}
            graphs = {k: v for k, v in graphs.items() if k in live}
    return (ranking.stat_ranks(ranks_raw, "raw_ent").item(), ranking.stat_ranks(ranks_filter, "filter_ent").item(),
            ranking.stat_ranks(ranks_raw_r, "raw_rel").item(), ranking.stat_ranks(ranks_filter_r, "filter_rel").item())


class GraphCache:
    """Device snapshot graphs keyed by the snapshot array's identity (built once, reused)."""

    def __init__(self, num_nodes, num_rels, device):
        self.n, self.r, self.dev, self.g = num_nodes, num_rels, device, {}

    def __call__(self, snap):
        key = id(snap)
        if key not in self.g:
            self.g[key] = (snap, build_sub_graph(self.n, self.r, snap, True, self.dev))
        return self.g[key][1]


def train_model(args, model, train_list, valid, num_nodes, num_rels, device, model_state_file):
    """hyperbolic_main.py:505-640 (`valid`: the validation rows with their time column).
    Returns {"best_mrr", "best_epoch", "epoch_loss": [mean loss per epoch]}."""
    import torch.distributed as dist
    from .parallel import allreduce_gradients
    world0 = dist.get_world_size() if dist.is_initialized() else 1
    if args.hip_graph and world0 > 1:
        logger.warning("--hip-graph is ignored with %d ranks: the replica step holds a gradient all-reduce "
                       "between its launches, so it runs eagerly", world0)
    if args.hip_graph and args.run_analysis:
        logger.warning("--hip-graph is ignored with --run-analysis: the analysis statistics are produced per "
                       "step on the host's schedule, so the steps run eagerly")
    graphed = GraphedSteps(device) if args.hip_graph and world0 == 1 and not args.run_analysis else None
    # :469; the fused multi-tensor kernel: a handful of launches per step instead of ~100 (it
    # does not bump the parameters' version counters: bump_versions after each step)
    fused = device.type == "cuda"
    optimizer = torch.optim.Adam(model.parameters(), lr=args.lr, weight_decay=1e-5,
                                 capturable=graphed is not None, fused=fused)
    # replicas: every rank takes its share of the shuffled samples, one gradient
    # all-reduce per optimizer step; the same seed on every rank keeps the shuffles (and so the
    # lock-step schedule) identical.  Rank 0 validates and checkpoints.
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    valid_list = ranking.split_by_time(valid)
    all_ans_v = ranking.load_all_answers_for_time_filter(valid, num_rels, num_nodes, False)
    all_ans_r_v = ranking.load_all_answers_for_time_filter(valid, num_rels, num_nodes, True)
    graphs = GraphCache(num_nodes, num_rels, device)
    tcache = {}

    def triple_cache(n):  # device triples per training snapshot, kept (a captured step reads them)
        if n not in tcache:
            tcache[n] = torch.from_numpy(np.asarray(train_list[n], dtype=np.int64)).to(device)
        return tcache[n]

    best_mrr, best_epoch, patience = 0.0, 0, 20
    epoch_loss = []
    valid_history = []  # (epoch, raw MRR, filtered MRR, raw rel MRR, filtered rel MRR) per validation
    summaries = []  # --run-analysis: get_training_summary() per epoch
    t_start = time.time()
    initial_curvature = None
    for epoch in range(args.n_epochs):
        t0 = time.time()
        model.train()
        if args.learn_curvature:  # hyperbolic_main.py:528-544: the upper bound warms up linearly
            if initial_curvature is None:
                initial_curvature = min(max(model.get_curvature().item(), args.curvature_min), args.curvature_max)
            if args.curvature_warmup_epochs > 0 and epoch < args.curvature_warmup_epochs:
                cmax = initial_curvature + (args.curvature_max - initial_curvature) * \
                    (epoch + 1) / args.curvature_warmup_epochs
            else:
                cmax = args.curvature_max
            model.set_curvature_bounds(curvature_max=cmax)
            if args.plus_relation_specific_curvature:
                model.set_relation_curvature_bounds(curvature_max=cmax)
        # per-sample losses accumulated on the device (the reference's four .item() per
        # mini-batch, :600-603, would synchronise every step): one read per epoch
        acc = torch.zeros(4, device=device, dtype=torch.float64)  # sum of e, r, rad; samples
        idx = list(range(len(train_list)))
        random.shuffle(idx)
        idx = [n for n in idx if n != 0 and len(train_list[n])]
        if args.max_train_snapshots:
            idx = idx[:args.max_train_snapshots]
        if world > 1:  # lock-step: every rank one sample per step
            idx = idx[:len(idx) // world * world][rank::world]
        for n in idx:
            inputs = train_list[max(0, n - args.train_history_len):n]
            glist = [graphs(s) for s in inputs]
            if not len(train_list[n]):
                continue
            triples = triple_cache(n)

            def step():
                optimizer.zero_grad()
                if args.reuse_encoder and hasattr(model, "get_loss_batches"):
                    # one encoder forward/backward per snapshot, the mini-batch losses summed
                    # (the decoders run once over all the snapshot's mini-batches inside)
                    parts = model.get_loss_batches(
                        glist, triples, None, True, args.triple_batch_size, query_time=n,
                        combine=lambda le, lr, ls, lrad: args.task_weight * le + (1 - args.task_weight) * lr
                        + ls.sum() + lrad)
                else:  # hyperbolic_main.py:585-598: the encoder recomputed per mini-batch
                    parts = []
                    for b in range(0, triples.shape[0], args.triple_batch_size):
                        le, lr, ls, lrad = model.get_loss(glist, triples[b:b + args.triple_batch_size], None, True,
                                                          query_time=n)
                        loss = args.task_weight * le + (1 - args.task_weight) * lr + ls.sum() + lrad
                        loss.backward()
                        parts.append((le, lr, ls, lrad))
                allreduce_gradients(model.parameters())
                if args.run_analysis and n % 100 == 0 and hasattr(model, "log_gradient_stats"):   # :623-625
                    model.log_gradient_stats()
                torch.nn.utils.clip_grad_norm_(model.parameters(), args.grad_norm)          # :627-628
                optimizer.step()
                if fused:  # the fused step leaves the version counters the caches key on
                    bump_versions(model.parameters())
                # the sample's mean mini-batch losses (entity, relation, radius)
                return torch.stack([torch.stack([p[k].detach().double() for p in parts]).mean() for k in (0, 1, 3)])

            means = graphed.run(n, step) if graphed is not None else step()
            acc[:3] += means
            acc[3] += 1
        tot = acc.cpu().numpy()
        if tot[3] > 0:
            me, mr, mrad = tot[:3] / tot[3]
            epoch_loss.append(float(args.task_weight * me + (1 - args.task_weight) * mr + mrad))
        else:
            me = mr = mrad = float("nan")
            epoch_loss.append(float("nan"))
        if epoch % args.log_interval == 0:
            logger.info("Epoch %04d | Loss: %.4f | E/R/S/Rad: %.4f/%.4f/%.4f/%.4f | Best MRR: %.4f | Time: %.1fs",
                        epoch, epoch_loss[-1], me, mr, 0.0, mrad, best_mrr, time.time() - t0)
        if args.run_analysis:                                                                # :617-621
            logger.debug("Radius loss: %.4f", mrad)
            if hasattr(model, "get_training_summary"):                                    # :655-657
                summary = model.get_training_summary()
                summaries.append(summary)
                logger.info("Training summary: %s", summary)
        if epoch and epoch % args.evaluate_every == 0:                                      # :660-681
            stop = torch.zeros(1, device=device)
            if rank == 0:
                if graphed is not None:
                    # a replay updates the parameters on the device without bumping their
                    # version counters: drop every parameter-keyed cache (packed weights,
                    # initial state, memo) so validation scores the current weights
                    invalidate(model)
                res = test(model, train_list, valid_list, num_rels, num_nodes, device, all_ans_v, all_ans_r_v, args)
                valid_history.append((epoch,) + tuple(float(v) for v in res))
                logger.info("Validation - MRR: raw=%.4f, filter=%.4f | Rel MRR: raw=%.4f, filter=%.4f", *res)
                cur = res[2] if args.relation_evaluation else res[0]
                if cur > best_mrr:
                    best_mrr, best_epoch = cur, epoch
                    os.makedirs(os.path.dirname(os.path.abspath(model_state_file)), exist_ok=True)
                    torch.save({"state_dict": model.state_dict(), "epoch": epoch}, model_state_file)
                    logger.info("New best model saved! MRR: %.4f", best_mrr)
                elif epoch - best_epoch >= patience:
                    logger.info("Early stopping at epoch %d: no improvement in %d epochs.", epoch, patience)
                    stop.fill_(1.0)
            if world > 1:
                dist.broadcast(stop, 0)
            if float(stop) > 0:
                break
    logger.info("Training completed in %.1f minutes", (time.time() - t_start) / 60)
    return {"best_mrr": best_mrr, "best_epoch": best_epoch, "epoch_loss": epoch_loss, "valid": valid_history,
            "summaries": summaries}


def main(argv=None):
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if args.verbose else logging.INFO, format="%(message)s")
    bad = _unsupported(args)
    if bad:
        raise SystemExit("not supported in this build (SURVEY.md §2 out of scope): " + ", ".join(bad))
    if args.curvature_warmup_epochs < 0:
        raise ValueError("curvature_warmup_epochs must be non-negative")          # hyperbolic_main.py:212-213
    if not args.test and args.hip_graph and args.learn_curvature:
        raise SystemExit("--hip-graph with --learn-curvature: the curvature changes every step and the "
                         "step reads it on the host (as the reference's c.item()); train it without --hip-graph")
    if args.radius_msg_gamma < 0:
        raise ValueError("--radius-msg-gamma must be non-negative (use 0 to disable the penalty)")
    if not 0.0 <= args.radius_anchor_beta <= 1.0:
        raise ValueError("--radius-anchor-beta must be in [0, 1]")
    if args.gpu < 0 or not torch.cuda.is_available():
        raise SystemExit("the HIP path needs a GPU (--gpu N); there is no CPU fallback")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        # one process per GPU (torchrun); replicas train on different snapshots and
        # all-reduce gradients over RCCL
        import torch.distributed as dist
        args.gpu = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(args.gpu)
        if not dist.is_initialized():
            backend = os.environ.get("REGCN_DIST_BACKEND", "nccl")  # gloo: replicas sharing one GPU in tests
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", args.gpu))
            else:
                dist.init_process_group(backend)
        if args.seed is None:
            args.seed = 0  # identical shuffles on every rank keep the lock-step schedule
    device = torch.device("cuda", args.gpu)
    torch.cuda.set_device(device)
    if args.seed is not None:
        random.seed(args.seed)
        np.random.seed(args.seed)
        torch.manual_seed(args.seed)
    num_nodes, num_rels, train, valid, test_data = load_dataset(args)
    train_list = ranking.split_by_time(train)
    valid_list = ranking.split_by_time(valid)
    test_list = ranking.split_by_time(test_data)
    logger.info("Dataset %s: %d entities, %d relations, %d/%d/%d snapshots", args.dataset, num_nodes, num_rels,
                len(train_list), len(valid_list), len(test_list))
    all_ans = ranking.load_all_answers_for_time_filter(test_data, num_rels, num_nodes, False)
    all_ans_r = ranking.load_all_answers_for_time_filter(test_data, num_rels, num_nodes, True)
    model = build_model(args, num_nodes, num_rels, train_list, device)
    if world > 1:
        from .parallel import broadcast_state
        broadcast_state(model)
    model_state_file = args.checkpoint or os.path.join(
        "models", "%s-%s-%s.pth" % (args.dataset.replace(":", "_"), args.encoder, args.decoder))
    if not args.test:
        train_model(args, model, train_list, valid, num_nodes, num_rels, device, model_state_file)
        args.checkpoint = model_state_file if os.path.exists(model_state_file) else None
    sharded_test = world > 1 and args.shard != "none"
    if world > 1 and not sharded_test:  # the test pass runs on rank 0
        import torch.distributed as dist
        dist.barrier()
        rank = dist.get_rank()
        dist.destroy_process_group()
        if rank != 0:
            return True
    if args.checkpoint:
        ck = torch.load(args.checkpoint, map_location=device, weights_only=True)
        model.load_state_dict(ck["state_dict"] if "state_dict" in ck else ck)
        logger.info("Load Model: %s. Using best epoch: %s", args.checkpoint, ck.get("epoch", "?"))
    t0 = time.time()
    res = test(model, train_list + valid_list, test_list, num_rels, num_nodes, device, all_ans, all_ans_r, args)
    logger.info("MRR raw %.6f filter %.6f | relation raw %.6f filter %.6f | %.2f s", *res, time.time() - t0)
    if sharded_test:  # every rank took part in the partitioned test pass
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return res


if __name__ == "__main__":
    sys.exit(0 if main() else 1)
