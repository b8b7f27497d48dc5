"""Device-time attribution of torch ops in one headline step: python scripts/torchprof_bench.py OUT.txt <bench args>
(torch.profiler with input shapes; the native HIP kernels show up under their own names)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

out = sys.argv[1]
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402

acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
    bench.main()
with open(out, "w") as f:
    ka = prof.key_averages(group_by_input_shape=True)
    f.write(ka.table(sort_by="self_cuda_time_total", row_limit=45, max_name_column_width=60,
                     max_shapes_column_width=90))
