"""Application entry point (``core/.../op/OpApp.scala:49-213``).

Subclass :class:`OpAppWithRunner` and implement :meth:`runner`; ``main(argv)`` parses the reference's
flags (``-t/--run-type``, ``-r/--read-location name=path``, ``-m/--model-location``, ``-w/--write-location``,
``-x/--metrics-location``, ``-p/--param-location``), merges them over the params file and dispatches
to :class:`~transmogrifai_amd.workflow.runner.OpWorkflowRunner`. Multi-GPU jobs start one process per
GPU (``torchrun``); every rank runs ``main`` and the process group is initialized from the env.
"""
from __future__ import annotations

import argparse
import sys
from typing import Optional, Sequence

from .workflow.params import OpParams
from .workflow.runner import OpWorkflowRunner, OpWorkflowRunnerConfig, OpWorkflowRunType


def parse_args(argv: Sequence[str], app_name: str = "op-app") -> OpWorkflowRunnerConfig:
    ap = argparse.ArgumentParser(prog=app_name)
    ap.add_argument("-t", "--run-type", required=True,
                    help="the type of workflow run: " + " | ".join(v.lower() for v in OpWorkflowRunType.values))
    ap.add_argument("-p", "--param-location", default=None, help="path to a json / yaml OpParams file")
    ap.add_argument("-r", "--read-location", action="append", default=[],
                    help="reader name=path (repeatable)")
    ap.add_argument("-m", "--model-location", default=None)
    ap.add_argument("-w", "--write-location", default=None)
    ap.add_argument("-x", "--metrics-location", default=None)
    a = ap.parse_args(list(argv))
    reads = {}
    for r in a.read_location:
        if "=" not in r:
            raise SystemExit(f"read location must be name=path, got {r}")
        k, v = r.split("=", 1)
        reads[k] = v
    return OpWorkflowRunnerConfig(OpWorkflowRunType.with_name_insensitive(a.run_type), OpParams(),
                                  a.param_location, reads, a.write_location, a.model_location, a.metrics_location)


class OpApp:
    app_name = "op-app"

    def run(self, run_type: str, params: OpParams):
        raise NotImplementedError

    def main(self, argv: Optional[Sequence[str]] = None):
        from .parallel import dist as D
        D.init_from_env()
        cfg = parse_args(sys.argv[1:] if argv is None else argv, self.app_name)
        params = cfg.to_op_params()
        cfg.validate(params)
        from .utils.device_errors import run_main
        return run_main(lambda: self.run(cfg.run_type, params), self.app_name)


class OpAppWithRunner(OpApp):
    def runner(self, params: OpParams) -> OpWorkflowRunner:
        raise NotImplementedError

    def run(self, run_type: str, params: OpParams):
        return self.runner(params).run(run_type, params)
