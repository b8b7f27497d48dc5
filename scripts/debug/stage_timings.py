"""Per-stage wall-clock breakdown of one headline AutoML train (bench.py config) on cuda:0.

Usage: python scripts/debug/stage_timings.py [rows]
Prints the workflow's OpStep / per-stage timings and the model selector's per-learner timings."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from transmogrifai_amd import config as CFG, uid
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.readers.base import InMemoryReader
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.testkit.synthetic import binary_table
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    dev = torch.device("cuda:0")
    CFG.set_default_device(dev)
    for it in range(2):
        uid.reset(0)
        ds, label, preds = binary_table(rows, 170, 15, 15, seed=7, device=dev)
        vec = transmogrify(preds)
        checked = label.sanity_check(vec, remove_bad_features=True)
        pred = BinaryClassificationModelSelector.with_cross_validation(num_folds=3, seed=42).set_input(
            label, checked).get_output()
        wf = OpWorkflow().set_result_features(label, pred).set_reader(InMemoryReader(ds))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model = wf.train()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        summ = model.get_origin_stage_of(pred).metadata["summary"]
        print(json.dumps({"iter": it, "total_s": dt, "timings": model.train_timings,
                          "selector": summ.get("timings")}, default=float), flush=True)


if __name__ == "__main__":
    main()
