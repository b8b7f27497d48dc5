"""``python -m transmogrifai_amd.cli gen --input data.csv --response y --id id --name Proj [--kind binary]``."""
from __future__ import annotations

import argparse
import sys


def main(argv=None):
    ap = argparse.ArgumentParser(prog="op")
    sub = ap.add_subparsers(dest="command", required=True)
    g = sub.add_parser("gen", help="generate a project from a data file")
    g.add_argument("--input", required=True, help="CSV with header, or avro file")
    g.add_argument("--response", required=True)
    g.add_argument("--id", required=True, dest="id_field")
    g.add_argument("--name", default="Sample")
    g.add_argument("--dest", default=".")
    g.add_argument("--schema", default=None, help="optional .avsc schema")
    g.add_argument("--kind", default=None, help="binary | multiclass | regression (inferred when omitted)")
    g.add_argument("--overwrite", action="store_true")
    a = ap.parse_args(argv)
    from .gen import generate
    d = generate(a.input, a.response, a.id_field, a.name, a.dest, a.kind, a.schema, a.overwrite)
    print(f"Project generated in {d}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
