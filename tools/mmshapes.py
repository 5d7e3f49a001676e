"""Shape census of the training step's GEMMs: torch profiler (input shapes) around a few
eager trainbench samples on the GPU; prints the matmul-family ops by device time."""
import sys, runpy, torch
from torch.profiler import profile, ProfilerActivity
sys.argv = ["trainbench", "--no-cpu", "--steps", "4", "--warmup", "1"]
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as p:
    runpy.run_path("tools/trainbench.py", run_name="__main__")
ka = p.key_averages(group_by_input_shape=True)
rows = [e for e in ka if any(k in e.key for k in ("mm", "linear", "matmul", "gru", "GRU"))]
rows.sort(key=lambda e: -e.device_time_total)
for e in rows[:40]:
    print(f"{e.key:28s} n={e.count:5d} dev_us={e.device_time_total/ max(1,e.count):8.1f} tot_ms={e.device_time_total/1e3:8.2f} {str(e.input_shapes)[:120]}")
