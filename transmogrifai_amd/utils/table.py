"""Plain-text table printer used by ``summary_pretty`` (``utils/.../utils/table/Table.scala``)."""
from __future__ import annotations

from typing import Dict, Optional, Sequence


def _fmt(v) -> str:
    if isinstance(v, float):
        return repr(v)
    return str(v)


def pretty_table(columns: Sequence[str], rows: Sequence[Sequence], name: str = "",
                 align: Optional[Dict[str, str]] = None) -> str:
    """Render ``rows`` under ``columns`` as a ``|---|`` bordered table.

    ``align`` maps a column name to ``"left"``, ``"right"`` or ``"center"`` (default left for the first
    column, right for the others, mirroring the reference ``Table.prettyString``).
    """
    align = align or {}
    cells = [[_fmt(c) for c in r] for r in rows]
    widths = [len(c) for c in columns]
    for r in cells:
        for i, c in enumerate(r):
            widths[i] = max(widths[i], len(c))
    sep = "|" + "|".join("-" * (w + 2) for w in widths) + "|"

    def cell(s, w, how):
        if how == "right":
            return s.rjust(w)
        if how == "center":
            return s.center(w)
        return s.ljust(w)

    head = "|" + "|".join(" " + c.center(w) + " " for c, w in zip(columns, widths)) + "|"
    out = []
    if name:
        out.append(sep)
        total = len(sep) - 4
        out.append("| " + name.center(total) + " |")
    out += [sep, head, sep]
    for r in cells:
        parts = []
        for i, (c, w) in enumerate(zip(r, widths)):
            how = align.get(columns[i], "left" if i == 0 else "right")
            parts.append(" " + cell(c, w, how) + " ")
        out.append("|" + "|".join(parts) + "|")
    out.append(sep)
    return "\n".join(out)
