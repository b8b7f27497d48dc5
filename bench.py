"""Headline benchmark: end-to-end AutoML train on a 10M-row binary-class synthetic table.

BASELINE.json metric: "end-to-end AutoML wall-clock + hold-out AuPR, 10M-row binary-class tabular".
One *step* is one complete ``OpWorkflow.train()``:

  raw columns (device resident) -> transmogrify() (RealVectorizer / IntegralVectorizer / one-hot pivot
  -> VectorsCombiner) -> SanityChecker(removeBadFeatures) -> BinaryClassificationModelSelector with
  3-fold CV over the reference default grid (LR x8, RF x18, XGBoost x2 = 84 CV fits), DataSplitter
  (10% hold-out reserve, 1M max training sample as in ``Splitter.scala:176-178``), refit of the
  winner, train + hold-out evaluation.

Multi-GPU (``torchrun``, one rank per GPU, RCCL over xGMI): each rank holds a contiguous row shard of
the table (``Dataset.shard``); transmogrify / SanityChecker fit statistics are all-reduced
(``parallel/dp.py``), the model selector gathers the rows its CV folds and refit sample (the 1M
``maxTrainingSample`` cap) to every rank and shards the (model, grid point, fold) fits across ranks by
a cost model (``tuning/validators.py``); the hold-out is scored on the local shard and its
(label, score) rows are all-gathered for the metrics. ``--layout replicated`` keeps the whole table on
every rank instead. Total work is fixed as N grows -> ``"scaling": "strong"``.

The value reported is the end-to-end wall-clock seconds of one AutoML train (lower is better); the
hold-out AuPR of the selected model is reported next to it. The reference publishes no wall-clock
 so ``vs_baseline`` is null.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "end-to-end AutoML wall-clock + hold-out AuPR, 10M-row binary-class tabular"

# BASELINE.json configs: name -> (metric, default rows, selector kind, hold-out metric key)
CONFIGS = {
    "binary-10m": (METRIC, 10_000_000, "binary", "AuPR"),
    "lr-rf-1m": ("end-to-end AutoML wall-clock + hold-out AuPR, 1M-row binary-class, LR + RandomForest selector",
                 1_000_000, "binary", "AuPR"),
    "multiclass-text": ("end-to-end AutoML wall-clock + hold-out error, multi-class tabular with text + categorical "
                        "columns (SmartText hashing-TF + one-hot)", 1_000_000, "multi", "Error"),
    "regression-100m": ("end-to-end AutoML wall-clock + hold-out RMSE, 100M-row regression, default regression "
                        "selector grid", 100_000_000, "regression", "RootMeanSquaredError"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="binary-10m", choices=sorted(CONFIGS),
                    help="BASELINE.json config: the headline (binary-10m) or one of the secondary configs")
    ap.add_argument("--rows", type=int, default=None, help="rows (default: the config's)")
    ap.add_argument("--real", type=int, default=170)
    ap.add_argument("--int", dest="ints", type=int, default=15)
    ap.add_argument("--pick", type=int, default=15)
    ap.add_argument("--models", default="default",
                    help="comma list of learner names, or 'default' (LR, RF, XGBoost as the reference)")
    ap.add_argument("--folds", type=int, default=3)
    ap.add_argument("--device", default=None)
    ap.add_argument("--layout", default="sharded", choices=["sharded", "replicated"],
                    help="multi-GPU table layout: row shards with all-reduced fit statistics (data parallel), "
                         "or the whole table on every rank")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--ingest", default="memory", choices=["memory", "parquet", "csv"],
                    help="memory: the device-resident synthetic table is the reader's input (the headline); parquet: "
                         "the table is written to a Parquet file before timing and every timed train reads it "
                         "(readers/columnar.py) inside the timed region")
    ap.add_argument("--ingest-dir", default=None, help="directory of the --ingest parquet file (default /tmp)")
    ap.add_argument("--max-training-sample", dest="max_training_sample", type=int, default=None,
                    help="the selector splitter's maxTrainingSample (default: the reference's 1M)")
    ap.add_argument("--dtype", default=None, choices=["fp32", "bf16"],
                    help="linear learners' design-matrix precision (config.linear_dtype): fp32 (default; the "
                         "headline's hold-out AuPR must equal the fp32 model's), or lossy bf16 on the bf16 matrix "
                         "cores (BASELINE config 2, lr-rf-1m '1 MI355X bf16'); tree learners bin their inputs "
                         "either way")
    a = ap.parse_args()
    if a.config == "lr-rf-1m" and a.models == "default":
        a.models = "OpLogisticRegression,OpRandomForestClassifier"
    if a.dtype is None:         # BASELINE.json names bf16 for config 2 only
        a.dtype = "bf16" if a.config == "lr-rf-1m" else "fp32"
    if a.rows is None:
        a.rows = CONFIGS[a.config][1]
    return a


def _rows_label(n: int) -> str:
    for div, suf in ((1_000_000, "M"), (1_000, "K")):
        if n % div == 0:
            return f"{n // div}{suf}-row"
    return f"{n}-row"


def _selector_cls(args):
    from transmogrifai_amd.selector import factories as F
    return {"binary": F.BinaryClassificationModelSelector, "multi": F.MultiClassificationModelSelector,
            "regression": F.RegressionModelSelector}[CONFIGS[args.config][2]]


def _expected_configs(args) -> int:
    """Grid points the selector must evaluate (default binary grid: LR 8 + RF 18 + XGBoost 2)."""
    types = None if args.models == "default" else args.models.split(",")
    sel = _selector_cls(args).with_cross_validation(num_folds=args.folds, model_types_to_use=types, seed=42)
    return sum(len(grid) for _, grid in sel.models)


def build_workflow(args, ds, label, preds, reader=None):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.readers.base import InMemoryReader
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    vec = transmogrify(preds)
    checked = label.sanity_check(vec, remove_bad_features=True)
    types = None if args.models == "default" else args.models.split(",")
    splitter = "default"
    if args.max_training_sample:
        splitter = _selector_cls(args)._default_splitter(42)
        splitter.max_training_sample = int(args.max_training_sample)
    pred = _selector_cls(args).with_cross_validation(
        splitter=splitter, num_folds=args.folds, model_types_to_use=types, seed=42).set_input(label, checked).get_output()
    wf = OpWorkflow().set_result_features(label, pred).set_reader(reader or InMemoryReader(ds))
    return wf, pred


def _spawned_rank(local_rank, n, port, argv):
    """Entry of a rank process started by ``bench.py --gpus N`` without torchrun."""
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(n),
                      LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.argv = argv
    main()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one rank per GPU, spawned before anything in this process touches the GPU (never exec)
        import torch.multiprocessing as mp
        mp.start_processes(_spawned_rank, args=(args.gpus, _free_port(), list(sys.argv)), nprocs=args.gpus,
                           join=True, start_method="spawn")
        return
    import torch
    from transmogrifai_amd import config as CFG
    from transmogrifai_amd.parallel import dist as D

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    use_gpu = args.device != "cpu" and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    else:
        dev = torch.device("cpu")
    sim = os.environ.get("TMOG_SIM_WORLD")
    if sim:      # projection (scripts/project_schedule.py): this process times rank TMOG_SIM_RANK's share
        # spread / hybrid learners run too: collectives are answered locally, and the tree grower's split-record
        # exchange is answered by tiling this rank's records (tree_grow_hip.hip tmog_hip_fp_allgather)
        D.simulate(int(os.environ.get("TMOG_SIM_RANK", "0")), int(sim))
    else:
        D.init_from_env(device_id=local_rank if use_gpu else None)
    world = D.world()
    if world != max(1, args.gpus) and args.device != "cpu" and not sim:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the process group has {world} ranks")
    CFG.set_default_device(dev)
    CFG.set_linear_dtype(args.dtype)
    if use_gpu:
        from transmogrifai_amd.ops import _native
        _native.hip()   # fail loudly if the HIP kernels cannot be loaded

    from transmogrifai_amd.testkit import synthetic as SY
    from transmogrifai_amd import uid

    def make_table():
        if args.config == "multiclass-text":
            return SY.multiclass_text_table(args.rows, seed=11, device=dev)
        if args.config == "regression-100m":
            return SY.regression_table(args.rows, seed=13, device=dev)
        return SY.binary_table(args.rows, args.real, args.ints, args.pick, seed=7, device=dev)

    def sync():
        if use_gpu:
            torch.cuda.synchronize()
        D.barrier()

    n_raw = [0]
    stage_t = [{}]
    # time the interpreter spends in garbage collection inside each timed train (per-step diagnostics)
    import gc
    gc_t = [0.0, None]

    def _gc_cb(phase, info):
        if phase == "start":
            gc_t[1] = time.perf_counter()
        elif gc_t[1] is not None:
            gc_t[0] += time.perf_counter() - gc_t[1]
            gc_t[1] = None

    gc.callbacks.append(_gc_cb)
    gc_steps = []

    pq_path = [None]

    def one_run():
        uid.reset(0)
        ds, label, preds = make_table()
        n_raw[0] = len(preds)
        if world > 1 and args.layout == "sharded":
            ds = ds.shard(D.rank(), world)      # N / world rows per GPU; global row ids kept
            if use_gpu:
                torch.cuda.empty_cache()
        reader = None
        if args.ingest in ("parquet", "csv"):
            from transmogrifai_amd.readers.columnar import dataset_to_csv, dataset_to_parquet
            from transmogrifai_amd.readers.files import CSVReader, ParquetReader
            if pq_path[0] is None:              # written once, untimed; the same seeded table every run
                d = args.ingest_dir or "/tmp"
                pq_path[0] = os.path.join(d, f"tmog_bench_{args.config}_{args.rows}_{os.getpid()}.{args.ingest}")
                t_w = time.perf_counter()
                (dataset_to_parquet if args.ingest == "parquet" else dataset_to_csv)(
                    ds, pq_path[0], names=[f.name for f in [label] + list(preds)])
                print(f"[ingest] wrote {pq_path[0]} ({os.path.getsize(pq_path[0]) / 1e9:.2f} GB) in "
                      f"{time.perf_counter() - t_w:.1f} s", file=sys.stderr, flush=True)
            reader = ParquetReader(pq_path[0], device=dev) if args.ingest == "parquet" else \
                CSVReader(pq_path[0], has_header=True, device=dev)
            if args.ingest == "csv":
                # the file holds this table's float32 reals as shortest float32 decimals: stored as float32 they
                # read back bit-identical to the in-memory table (Parquet keeps the float32 type itself)
                reader.real_dtype = torch.float32
            del ds
            ds = None
            if use_gpu:
                torch.cuda.empty_cache()
        wf, pred = build_workflow(args, ds, label, preds, reader)
        sync()
        gc_t[0] = 0.0
        t0 = time.perf_counter()
        model = wf.train()
        sync()
        dt = time.perf_counter() - t0
        gc_steps.append(round(gc_t[0], 4))
        stage_t[0] = {k: round(v, 4) for k, v in model.train_timings.items() if isinstance(v, (int, float))}
        per_stage = model.train_timings.get("stages", {})
        stage_t[0]["top_stages"] = dict(sorted(((k, round(v, 4)) for k, v in per_stage.items()
                                                if isinstance(v, (int, float)) and not k.startswith("peak_gb")),
                                               key=lambda kv: -kv[1])[:12])
        sel = model.get_origin_stage_of(pred)
        summ = sel.metadata.get("summary", {})
        ho = (summ.get("holdoutEvaluation") or {}).get(CONFIGS[args.config][3], float("nan"))
        # a learner that dies must not make the headline faster: every configured grid point must have
        # been evaluated and nothing may have failed
        n_eval = len(summ.get("validationResults") or [])
        if summ.get("failures") or (n_eval != expected_configs and not sim):   # (a simulated rank sees its share)
            raise SystemExit(f"model selector evaluated {n_eval}/{expected_configs} configs; failures: "
                             f"{summ.get('failures')}")
        if os.environ.get("TMOG_MEM_TRACE") == "1" and D.rank() == 0:
            st = model.train_timings.get("stages", {})
            print(json.dumps({k: v for k, v in st.items() if k.startswith("peak_gb")}), flush=True)
        return dt, ho, summ

    expected_configs = _expected_configs(args)
    if args.ingest != "memory" and world > 1:
        raise SystemExit("--ingest parquet / csv is a single-GPU measurement")
    try:
        _timed(args, one_run, expected_configs, use_gpu, dev, torch, D, sim, n_raw, stage_t, gc_steps, world)
    finally:
        if pq_path[0] and os.path.exists(pq_path[0]):
            os.remove(pq_path[0])
    if D.is_dist() and not sim:
        import torch.distributed as dist
        dist.destroy_process_group()


def _timed(args, one_run, expected_configs, use_gpu, dev, torch, D, sim, n_raw, stage_t, gc_steps, world):
    for _ in range(args.warmup):
        one_run()
    if use_gpu:
        torch.cuda.reset_peak_memory_stats(dev)
    times, auprs, summ = [], [], None
    for _ in range(args.steps):
        dt, ho, summ = one_run()
        times.append(dt)
        auprs.append(ho)
    t = torch.tensor([sum(times)], dtype=torch.float64)
    t = D.all_reduce(t, "max")
    total = float(t.item())
    peak = torch.tensor([float(torch.cuda.max_memory_allocated(dev)) if use_gpu else 0.0], dtype=torch.float64)
    peak = float(D.all_reduce(peak, "max").item())
    from transmogrifai_amd.parallel import dp as DP
    _all_fallbacks = [x for part in (D.all_gather_object(list(DP.GATHER_FALLBACKS)) if D.is_dist()
                                     else [DP.GATHER_FALLBACKS]) for x in part]
    per_step = total / max(args.steps, 1)
    if D.rank() == 0 or sim:
        metric = CONFIGS[args.config][0]
        if args.rows != CONFIGS[args.config][1]:       # the metric names the row count it was measured on
            metric = metric.replace(_rows_label(CONFIGS[args.config][1]), _rows_label(args.rows))
        out = {
            "metric": metric,
            "value": per_step,
            "unit": "s per end-to-end AutoML train",
            "n_gpus": world if use_gpu else 0,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1000.0,
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.dtype if use_gpu else "fp32",     # the bf16 design is a device path
            "data": "synthetic (device-generated, seeded), random-init models",
            ("holdout_aupr" if CONFIGS[args.config][3] == "AuPR" else
             "holdout_" + CONFIGS[args.config][3].lower()): auprs[-1],
            "best_model": summ.get("bestModelType") if summ else None,
            "configs_evaluated": len(summ.get("validationResults") or []) if summ else 0,
            "peak_hbm_gb_per_gpu": round(peak / 1e9, 3),
            "dp_gather_fallbacks": sorted(set(_all_fallbacks)),
            "schedule": {k: v[0] if v[0] != "hybrid" else f"hybrid:{v[3]}" for k, v in
                         (summ.get("schedule") or {}).items()} if summ else {},
            "config": {"name": args.config,
                       "model": _selector_cls(args).__name__ + "(" +
                                ("default grid" if args.models == "default" else args.models) + ")",
                       "rows": args.rows, "raw_columns": n_raw[0],
                       "cv_folds": args.folds, "global_batch": args.rows, "seq_len": None,
                       "max_training_sample": args.max_training_sample or 1_000_000,
                       "parallelism": (f"dp{world}" if args.layout == "sharded" else f"grid-shard{world}")
                       if world > 1 else "single"},
        }
        out["step_s"] = [round(x, 4) for x in times]
        out["gc_s"] = gc_steps[-len(times):] if times else []
        from transmogrifai_amd.utils import watchdog as WD
        if WD.STALLS:                                   # fit-progress stalls seen by the lanes watchdog
            out["stalls"] = list(WD.STALLS)
        if args.verbose and summ:
            out["timings"] = summ.get("timings")
            from transmogrifai_amd.tuning.validators import PHASE_TIMES
            if PHASE_TIMES:         # TMOG_FIT_PHASES=1, summed over the warm-up and timed steps
                out["fit_phases"] = {k: round(v, 4) for k, v in PHASE_TIMES.items()}
            out["stage_timings"] = stage_t[0]
        if sim:
            out["simulated"] = {"rank": D.rank(), "world": D.world(),
                                "note": "one rank's share timed on one GPU; collectives not executed"}
        if args.ingest != "memory":
            out["config"]["ingest"] = args.ingest
            out["data"] = (f"synthetic (device-generated, seeded), written to a {args.ingest} file before timing and "
                           "read by every timed train (readers/columnar.py), random-init models")
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    from transmogrifai_amd.utils.device_errors import run_main
    run_main(main, "bench.py")
