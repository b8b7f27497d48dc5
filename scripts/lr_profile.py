"""Host profile of one learner's model selection (python scripts/lr_profile.py [config] [learner] [rows]): the
bench workflow with that learner only, trained twice on the device; the second train under cProfile, sorted by
cumulative time (device waits show up in the calls that synchronise: .item(), .tolist(), bool(tensor))."""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from transmogrifai_amd import config as CFG, uid  # noqa: E402
from transmogrifai_amd.testkit import synthetic as SY  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "multiclass-text"
    learner = sys.argv[2] if len(sys.argv) > 2 else "OpLogisticRegression"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else bench.CONFIGS[cfg][1]
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    CFG.set_default_device(dev)
    CFG.set_linear_dtype("bf16")
    if dev.type == "cuda":
        from transmogrifai_amd.ops import _native
        _native.hip()
    if cfg == "multiclass-text":
        ds, label, preds = SY.multiclass_text_table(n, seed=11, device=dev)
    else:
        ds, label, preds = SY.binary_table(n, 170, 15, 15, seed=7, device=dev)
    args = argparse.Namespace(config=cfg, models=learner, folds=3, max_training_sample=None)

    def run():
        uid.reset(0)
        wf, _ = bench.build_workflow(args, ds, label, preds)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t = time.perf_counter()
        m = wf.train()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        print(f"train {time.perf_counter() - t:.3f} s", flush=True)
        return m

    run()
    pr = cProfile.Profile()
    pr.enable()
    run()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
    print(s.getvalue()[:9000])
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue()[:6000])


if __name__ == "__main__":
    main()
