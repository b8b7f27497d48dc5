"""``op gen``: generate a runnable AutoML project from a data file (``cli/.../gen/*.scala``).

Reference: ``CliParameters`` / ``CommandParser`` (``cli/.../CliExec.scala:81-83``), ``ProblemSchema.from``
(response field -> problem kind, id field, raw features from the Avro schema), ``ProblemKind``
(binary / multiclass / regression, asked when it cannot be inferred) and the project templates
(``cli/.../gen/templates``). The generated project is a Python package with an ``OpAppWithRunner``
whose workflow is ``transmogrify -> sanity_check -> <Kind>ModelSelector``, plus a params file and a
README with the train / score / evaluate commands.

Schemas come from a CSV header (types inferred with pandas), an Avro container file or an ``.avsc``.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import textwrap
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

BINARY, MULTI, REGRESSION = "BinaryClassification", "MultiClassification", "Regression"
KIND_ALIASES = {"binclass": BINARY, "binary classification": BINARY, "binary": BINARY,
                "multiclass": MULTI, "multi classification": MULTI, "regress": REGRESSION,
                "regression": REGRESSION}


@dataclass
class Field:
    name: str
    kind: str          # "real" | "integral" | "binary" | "text" | "categorical"
    nullable: bool = True


def _avro_kind(t) -> Tuple[str, bool]:
    nullable = False
    if isinstance(t, list):
        nullable = "null" in t
        t = next((x for x in t if x != "null"), "null")
    if isinstance(t, dict):
        t = t.get("type")
    return {"double": "real", "float": "real", "int": "integral", "long": "integral", "boolean": "binary",
            "string": "text", "enum": "categorical"}.get(t, "text"), nullable


def fields_from_avro(schema: dict) -> List[Field]:
    out = []
    for f in schema["fields"]:
        k, n = _avro_kind(f["type"])
        out.append(Field(f["name"], k, n))
    return out


def fields_from_frame(df, max_categorical: int = 30) -> List[Field]:
    import pandas as pd
    out = []
    for c in df.columns:
        s = df[c]
        nullable = bool(s.isna().any())
        if pd.api.types.is_bool_dtype(s):
            k = "binary"
        elif pd.api.types.is_integer_dtype(s):
            k = "integral"
        elif pd.api.types.is_float_dtype(s):
            k = "real"
        else:
            k = "categorical" if s.nunique(dropna=True) <= max_categorical else "text"
        out.append(Field(str(c), k, nullable))
    return out


def load_schema(input_file: str, schema_file: Optional[str] = None) -> Tuple[List[Field], str]:
    """(fields, reader kind) for a CSV with header, an avro file or an avsc schema."""
    from ..readers.avro import read_avro_schema
    if schema_file:
        return fields_from_avro(read_avro_schema(schema_file)), "avro" if input_file.endswith(".avro") else "csv"
    if input_file.endswith(".avro"):
        return fields_from_avro(read_avro_schema(input_file)), "avro"
    import pandas as pd
    df = pd.read_csv(input_file, nrows=10000)
    return fields_from_frame(df), "csv"


def infer_kind(input_file: str, response: Field, reader: str) -> Optional[str]:
    """Infer the problem kind from the response values; None when ambiguous (then the user is asked)."""
    import pandas as pd
    if reader == "avro":
        from ..readers.avro import read_avro
        vals = pd.Series([r.get(response.name) for r in read_avro(input_file)[:10000]])
    else:
        vals = pd.read_csv(input_file, usecols=[response.name], nrows=10000)[response.name]
    u = vals.dropna().unique()
    if response.kind == "binary" or len(u) == 2:
        return BINARY
    if response.kind in ("categorical", "text") or (response.kind == "integral" and len(u) <= 20):
        return MULTI if len(u) > 2 else BINARY
    if response.kind == "real":
        return REGRESSION
    return None


_TYPE = {"real": "Real", "integral": "Integral", "binary": "Binary", "text": "Text", "categorical": "PickList"}
_SELECTOR = {BINARY: "BinaryClassificationModelSelector", MULTI: "MultiClassificationModelSelector",
             REGRESSION: "RegressionModelSelector"}
_EVALUATOR = {BINARY: "Evaluators.BinaryClassification()", MULTI: "Evaluators.MultiClassification()",
              REGRESSION: "Evaluators.Regression()"}


def _ident(name: str) -> str:
    s = re.sub(r"\W+", "_", name).strip("_").lower() or "f"
    return "f_" + s if s[0].isdigit() else s


def render_app(proj: str, fields: List[Field], response: Field, id_field: str, kind: str, reader: str,
               data_path: str) -> str:
    resp_type = "RealNN"
    lines = []
    for f in fields:
        if f.name in (response.name, id_field):
            continue
        lines.append(f'    {_ident(f.name)} = FeatureBuilder.{_TYPE[f.kind]}("{f.name}").as_predictor()')
    feats = ", ".join(_ident(f.name) for f in fields if f.name not in (response.name, id_field))
    if kind == REGRESSION or response.kind in ("real", "integral", "binary"):
        resp_def = (f'    {_ident(response.name)} = FeatureBuilder.{resp_type}("{response.name}")'
                    f'.extract(response_value).as_response()')
    else:
        resp_def = (f'    {_ident(response.name)} = FeatureBuilder.{resp_type}("{response.name}")'
                    f'.extract(response_index).as_response()')
    reader_expr = (f'DataReaders.Simple.avro(path, key=record_key)' if reader == "avro" else
                   f'DataReaders.Simple.csv_auto(path, key=record_key)')
    r = _ident(response.name)
    return f'''"""{proj}: generated by `python -m transmogrifai_amd.cli gen` ({kind}).

Train:    python -m {proj.lower()}.app -t train -r data={data_path} -m model -x metrics
Score:    python -m {proj.lower()}.app -t score -r data={data_path} -m model -w scores
Evaluate: python -m {proj.lower()}.app -t evaluate -r data={data_path} -m model -x metrics
"""
from transmogrifai_amd.app import OpAppWithRunner
from transmogrifai_amd.dsl import transmogrify
from transmogrifai_amd.evaluators.evaluators import Evaluators
from transmogrifai_amd.features.builder import FeatureBuilder
from transmogrifai_amd.readers.files import DataReaders
from transmogrifai_amd.selector.factories import {_SELECTOR[kind]}
from transmogrifai_amd.workflow.runner import OpWorkflowRunner
from transmogrifai_amd.workflow.workflow import OpWorkflow

LABELS = {{}}


def record_key(r):
    return str(r.get("{id_field}"))


def response_value(r):
    v = r.get("{response.name}")
    return None if v is None or v != v else float(v)


def response_index(r):
    v = r.get("{response.name}")
    return float(LABELS.setdefault(str(v), len(LABELS)))


def build():
{resp_def}
{chr(10).join(lines)}
    features = transmogrify([{feats}])
    checked = {r}.sanity_check(features, remove_bad_features=True)
    prediction = {_SELECTOR[kind]}.with_cross_validation().set_input({r}, checked).get_output()
    evaluator = {_EVALUATOR[kind]}.set_label_col({r}).set_prediction_col(prediction)
    return OpWorkflow().set_result_features({r}, prediction), evaluator


class App(OpAppWithRunner):
    app_name = "{proj}"

    def runner(self, params):
        workflow, evaluator = build()
        rp = next(iter(params.reader_params.values()), None)
        path = rp.path if rp is not None else "{data_path}"
        reader = {reader_expr}
        return OpWorkflowRunner(workflow, training_reader=reader, scoring_reader=reader,
                                evaluation_reader=reader, evaluator=evaluator,
                                scoring_evaluator=evaluator, app_name="{proj}")


if __name__ == "__main__":
    App().main()
'''


def generate(input_file: str, response: str, id_field: str, proj_name: str = "Sample", location: str = ".",
             kind: Optional[str] = None, schema_file: Optional[str] = None, overwrite: bool = False,
             answers: Optional[Dict[str, str]] = None) -> str:
    """Write the project; returns its directory."""
    fields, reader = load_schema(input_file, schema_file)
    names = [f.name for f in fields]
    if response not in names:
        raise ValueError(f"Response field '{response}' not found in schema: {names}")
    if id_field not in names:
        raise ValueError(f"Id field '{id_field}' not found in schema: {names}")
    resp = next(f for f in fields if f.name == response)
    k = KIND_ALIASES.get(str(kind).lower(), kind) if kind else infer_kind(input_file, resp, reader)
    if k is None:
        ans = (answers or {}).get("kind")
        if ans is None:
            raise ValueError(f"Cannot infer the kind of problem based on response field '{response}'. "
                             f"Pass kind= one of {sorted(KIND_ALIASES)}")
        k = KIND_ALIASES[ans.lower()]
    pdir = os.path.join(location, proj_name.lower())
    if os.path.exists(pdir):
        if not overwrite:
            raise FileExistsError(f"Directory '{pdir}' already exists (use overwrite)")
        shutil.rmtree(pdir)
    pkg = os.path.join(pdir, proj_name.lower())
    os.makedirs(pkg)
    with open(os.path.join(pkg, "__init__.py"), "w") as f:
        f.write("")
    with open(os.path.join(pkg, "app.py"), "w") as f:
        f.write(render_app(proj_name, fields, resp, id_field, k, reader, os.path.abspath(input_file)))
    params = {"stageParams": {}, "readerParams": {"data": {"path": os.path.abspath(input_file)}},
              "customParams": {"problemKind": k}}
    with open(os.path.join(pdir, "params.json"), "w") as f:
        json.dump(params, f, indent=2)
    with open(os.path.join(pdir, "README.md"), "w") as f:
        f.write(f"# {proj_name}\n\nGenerated {k} project over `{input_file}` (response `{response}`, "
                f"id `{id_field}`).\n\n```\ncd {pdir}\npython -m {proj_name.lower()}.app -t train -p params.json "
                f"-m model -x metrics\npython -m {proj_name.lower()}.app -t score -p params.json -m model -w scores\n"
                f"```\n")
    return pdir
