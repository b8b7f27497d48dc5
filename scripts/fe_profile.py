"""Feature-engineering profile of a BASELINE config (python scripts/fe_profile.py [config] [rows]): transmogrify +
SanityChecker fitted through OpWorkflow twice on the device; the second run under cProfile (host time per
function, device synchronised at stage boundaries by the workflow's stage timers) and torch.profiler (device time
per kernel)."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd import config as CFG, uid  # noqa: E402
from transmogrifai_amd.dsl import transmogrify  # noqa: E402
from transmogrifai_amd.readers.base import InMemoryReader  # noqa: E402
from transmogrifai_amd.testkit import synthetic as SY  # noqa: E402
from transmogrifai_amd.workflow.workflow import OpWorkflow  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "multiclass-text"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    CFG.set_default_device(dev)
    if dev.type == "cuda":
        from transmogrifai_amd.ops import _native
        _native.hip()
    if cfg == "multiclass-text":
        ds, label, preds = SY.multiclass_text_table(n, seed=11, device=dev)
    else:
        ds, label, preds = SY.binary_table(n, 170, 15, 15, seed=7, device=dev)

    def run():
        uid.reset(0)
        vec = transmogrify(preds)
        checked = label.sanity_check(vec, remove_bad_features=True)
        wf = OpWorkflow().set_result_features(label, checked).set_reader(InMemoryReader(ds))
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t = time.perf_counter()
        m = wf.train()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        st = m.train_timings.get("stages", {})
        top = sorted(((k, v) for k, v in st.items() if isinstance(v, float)), key=lambda kv: -kv[1])[:8]
        print(f"FE train {time.perf_counter() - t:.3f} s", {k: round(v, 4) for k, v in top}, flush=True)

    run()
    pr = cProfile.Profile()
    pr.enable()
    run()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue()[:7000])
    acts = [torch.profiler.ProfilerActivity.CPU] + ([torch.profiler.ProfilerActivity.CUDA] if dev.type == "cuda" else [])
    with torch.profiler.profile(activities=acts) as prof:
        run()
    print(prof.key_averages().table(sort_by="self_cuda_time_total" if dev.type == "cuda" else "self_cpu_time_total",
                                    row_limit=30, max_name_column_width=70))


if __name__ == "__main__":
    main()
