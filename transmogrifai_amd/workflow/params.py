"""Run configuration (``features/.../OpParams.scala:81-318``).

``stageParams`` maps a stage class simple name **or** uid to ``{param: value}``; they are injected
into matching stages by :meth:`OpWorkflow.set_parameters` (``OpWorkflow.scala:179-201``). Loads from
JSON or YAML (``yaml.safe_load`` only).
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, Optional


@dataclass
class ReaderParams:
    path: Optional[str] = None
    partitions: Optional[int] = None
    custom_params: Dict[str, Any] = field(default_factory=dict)

    def to_json(self):
        return {"path": self.path, "partitions": self.partitions, "customParams": self.custom_params}

    @staticmethod
    def from_json(d):
        return ReaderParams(d.get("path"), d.get("partitions"), dict(d.get("customParams", {}) or {}))


@dataclass
class OpParams:
    stage_params: Dict[str, Dict[str, Any]] = field(default_factory=dict)
    reader_params: Dict[str, ReaderParams] = field(default_factory=dict)
    model_location: Optional[str] = None
    write_location: Optional[str] = None
    metrics_location: Optional[str] = None
    metrics_compress: Optional[bool] = None
    metrics_codec: Optional[str] = None
    log_stage_metrics: Optional[bool] = None
    collect_stage_metrics: Optional[bool] = None
    custom_tag_name: Optional[str] = None
    custom_tag_value: Optional[str] = None
    custom_params: Dict[str, Any] = field(default_factory=dict)
    alternate_reader_params: Dict[str, ReaderParams] = field(default_factory=dict)

    def to_json(self) -> Dict[str, Any]:
        return {"stageParams": self.stage_params,
                "readerParams": {k: v.to_json() for k, v in self.reader_params.items()},
                "modelLocation": self.model_location, "writeLocation": self.write_location,
                "metricsLocation": self.metrics_location, "metricsCompress": self.metrics_compress,
                "metricsCodec": self.metrics_codec, "logStageMetrics": self.log_stage_metrics,
                "collectStageMetrics": self.collect_stage_metrics, "customTagName": self.custom_tag_name,
                "customTagValue": self.custom_tag_value, "customParams": self.custom_params,
                "alternateReaderParams": {k: v.to_json() for k, v in self.alternate_reader_params.items()}}

    def to_string(self) -> str:
        return json.dumps(self.to_json(), default=str)

    @staticmethod
    def from_json(d: Dict[str, Any]) -> "OpParams":
        return OpParams(
            stage_params=dict(d.get("stageParams", {}) or {}),
            reader_params={k: ReaderParams.from_json(v) for k, v in (d.get("readerParams") or {}).items()},
            model_location=d.get("modelLocation"), write_location=d.get("writeLocation"),
            metrics_location=d.get("metricsLocation"), metrics_compress=d.get("metricsCompress"),
            metrics_codec=d.get("metricsCodec"), log_stage_metrics=d.get("logStageMetrics"),
            collect_stage_metrics=d.get("collectStageMetrics"), custom_tag_name=d.get("customTagName"),
            custom_tag_value=d.get("customTagValue"), custom_params=dict(d.get("customParams", {}) or {}),
            alternate_reader_params={k: ReaderParams.from_json(v)
                                     for k, v in (d.get("alternateReaderParams") or {}).items()})

    @staticmethod
    def from_string(s: str) -> "OpParams":
        """JSON, else YAML (``yaml.safe_load``); anything that is not a mapping of params is a ValueError (the
        reference's ``Failure(IllegalArgumentException)``)."""
        try:
            d = json.loads(s)
        except json.JSONDecodeError:
            import yaml
            try:
                d = yaml.safe_load(s)
            except yaml.YAMLError as e:
                raise ValueError(f"OpParams: neither JSON nor YAML: {e}") from e
        if d is None:
            d = {}
        if not isinstance(d, dict):
            raise ValueError(f"OpParams: expected a mapping of parameters, got {type(d).__name__}")
        return OpParams.from_json(d)

    @staticmethod
    def from_file(path: str) -> "OpParams":
        with open(path) as f:
            return OpParams.from_string(f.read())

    def switch_reader_params(self) -> "OpParams":
        """``switchReaderParams`` (OpParams.scala:203): the alternate reader params become the main ones."""
        out = self.with_values()
        out.reader_params, out.alternate_reader_params = dict(self.alternate_reader_params), dict(self.reader_params)
        return out

    def with_values(self, read_locations: Optional[Dict[str, str]] = None,
                    alternate_read_locations: Optional[Dict[str, str]] = None, **kw) -> "OpParams":
        """``withValues`` (OpParams.scala:116-150): new read paths per reader (added or replacing the reader's
        path) and any of the location / flag fields."""
        out = self._with(**kw)

        def upd(rp, locs):
            rp = dict(rp)
            for k, path in (locs or {}).items():
                old = rp.get(k) or ReaderParams()
                rp[k] = ReaderParams(path, old.partitions, dict(old.custom_params))
            return rp
        out.reader_params = upd(self.reader_params, read_locations)
        out.alternate_reader_params = upd(self.alternate_reader_params, alternate_read_locations)
        return out

    def _with(self, **kw) -> "OpParams":
        d = asdict(self)
        d.update({k: v for k, v in kw.items() if v is not None})
        out = OpParams(**{k: v for k, v in d.items() if k not in ("reader_params", "alternate_reader_params")})
        out.reader_params = dict(self.reader_params)
        out.alternate_reader_params = dict(self.alternate_reader_params)
        return out
