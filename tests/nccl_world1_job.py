"""One-rank job of tests/test_gpu_sharded.py::test_rccl_device_branches_world1: the RCCL
(backend "nccl") branches of parallel._all_to_all_into / _all_gather_into, which no gloo test
reaches, driven on a side stream exactly as ShardedGraph.run_layer drives them (comm stream
waits on the compute stream, the collective runs inside torch.cuda.stream(comm), the compute
stream waits back), and the same calls over a gloo group of the same rank; the results must be
equal bit for bit.  With one rank an all_to_all sends a rank its own records and an all-gather
returns its own chunk, so the expected values are known without a second GPU.  Writes a JSON
summary to argv[1]."""
import json
import os
import sys

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "re-gcn_amd"))


def main(out_path):
    from regcn_amd import parallel as P
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    gloo = dist.new_group(backend="gloo")
    res = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    g = torch.Generator(device="cpu").manual_seed(5)
    V, d = 4096, 200
    x0 = torch.randn(V, d, generator=g).to(dev)
    r0 = torch.rand(V, generator=g).to(dev) + 0.5
    sidx = torch.randperm(V, generator=g)[:700].to(dev)  # the rows this rank sends (to itself)
    ridx = torch.randperm(V, generator=g)[:700].to(dev)  # where the received records land
    chunk = (sidx, [700], ridx, [700])
    cur = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev)
    outs = {}
    for name, grp in (("nccl", None), ("gloo", gloo)):
        xn, rn = x0.clone(), r0.clone()
        full = torch.zeros(3 * 512, d, device=dev)
        part = torch.randn(3 * 512, d, generator=g).to(dev)
        comm.wait_stream(cur)
        with torch.cuda.stream(comm):
            P.exchange_rows(chunk, xn, rn, grp)                     # all_to_all_single
            for j in range(3):                                      # in-place chunk all-gathers
                P._all_gather_into(full[j * 512:(j + 1) * 512], part[j * 512:(j + 1) * 512], grp)
        cur.wait_stream(comm)
        for t in (xn, rn, full, part):
            t.record_stream(comm)
        torch.cuda.synchronize()
        outs[name] = (xn, rn, full, part)
    want_x, want_r = x0.clone(), r0.clone()
    want_x[ridx] = x0[sidx]
    want_r[ridx] = r0[sidx]
    xn, rn, full, part = outs["nccl"]
    res["nccl_exchange_exact"] = bool(torch.equal(xn, want_x) and torch.equal(rn, want_r))
    res["nccl_allgather_exact"] = bool(torch.equal(full, part))
    res["nccl_equals_gloo"] = bool(all(torch.equal(a, b) for a, b in zip(outs["nccl"][:2], outs["gloo"][:2])))
    with open(out_path, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
