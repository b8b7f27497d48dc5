"""Projection of an N-GPU headline run from one GPU: every rank's share of the schedule is
timed in its own process with ``TMOG_SIM_WORLD=N TMOG_SIM_RANK=r`` (parallel/dist.py projection mode: the rank
generates the full table, keeps its 1/N row shard, and every collective returns what it would if all ranks held
identical shards -- no communication is executed). The per-rank critical path is the projected step time
WITHOUT communication; the collectives of the real run (small all-reduces per fit stage, the metric exchange,
the training-sample gather) are listed separately as an estimate.

python scripts/project_schedule.py --world 8 [--rows 10000000] [--steps 1] [--warmup 1] [--out gpurun_out/proj]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--ranks", default=None, help="comma list (default: all)")
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "proj"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    ranks = [int(r) for r in a.ranks.split(",")] if a.ranks else list(range(a.world))
    rows = []
    for r in ranks:
        env = dict(os.environ, TMOG_SIM_WORLD=str(a.world), TMOG_SIM_RANK=str(r))
        cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--rows", str(a.rows), "--steps", str(a.steps),
               "--warmup", str(a.warmup), "--verbose"]
        t0 = time.time()
        # the rank's output goes straight to its log file (progress visible while it runs)
        logp = os.path.join(a.out, f"rank{r}.log")
        with open(logp, "w") as f:
            p = subprocess.run(cmd, env=env, stdout=f, stderr=subprocess.STDOUT, text=True, timeout=a.timeout,
                               cwd=ROOT)
        with open(logp) as f:
            p.stdout = f.read()
        if p.returncode != 0:
            print(f"rank {r}: exit {p.returncode}; see {a.out}/rank{r}.log", flush=True)
            sys.exit(p.returncode)
        line = [l for l in p.stdout.splitlines() if l.startswith('{"metric"')][-1]
        d = json.loads(line)
        row = {"rank": r, "step_s": round(d["value"], 4), "wall_s": round(time.time() - t0, 1),
               "learners": {k: round(v, 4) for k, v in (d.get("timings") or {}).items()
                            if k in ("OpLogisticRegression", "OpRandomForestClassifier", "OpXGBoostClassifier")},
               "stages": {k: v for k, v in (d.get("stage_timings") or {}).items() if k != "top_stages"},
               "configs_evaluated": d.get("configs_evaluated")}
        rows.append(row)
        print(json.dumps(row), flush=True)
    crit = max(rows, key=lambda x: x["step_s"])
    summary = {"world": a.world, "rows": a.rows, "per_rank_step_s": [x["step_s"] for x in rows],
               "critical_path_s": crit["step_s"], "critical_rank": crit["rank"],
               "configs_total": sum(x["configs_evaluated"] or 0 for x in rows),
               "note": "projection: per-rank share timed on one GPU with collectives not executed "
                       "(parallel/dist.py simulate); communication excluded"}
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump({"summary": summary, "ranks": rows}, f, indent=1)
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
