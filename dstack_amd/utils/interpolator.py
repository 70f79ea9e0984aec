"""``${{ namespace.var }}`` interpolation (reference: ``utils/interpolator.py:19-84``).

Used for ``${{ secrets.NAME }}``, ``${{ env.NAME }}``, ``${{ run.args }}`` in configurations and
``${{ dstack.node_rank }}`` in volume names/paths.  ``$${{`` escapes a literal ``${{``.
"""

from __future__ import annotations

import re
from typing import Dict, List, Optional, Tuple

_RE = re.compile(r"\$?\$\{\{\s*([a-zA-Z_][a-zA-Z0-9_]*)\.([a-zA-Z_][a-zA-Z0-9_]*)\s*\}\}")


class InterpolatorError(ValueError):
    pass


class VariablesInterpolator:
    def __init__(self, namespaces: Dict[str, Dict[str, str]], skip: Optional[List[str]] = None):
        self.namespaces = namespaces
        self.skip = set(skip or [])

    def interpolate(self, s: str, return_missing: bool = False):
        missing: List[str] = []

        def repl(m: re.Match) -> str:
            text = m.group(0)
            if text.startswith("$$"):
                return text[1:]
            ns, name = m.group(1), m.group(2)
            if ns in self.skip:
                return text
            if ns not in self.namespaces:
                raise InterpolatorError(f"Unknown namespace `{ns}` in {text}")
            if name not in self.namespaces[ns]:
                missing.append(f"{ns}.{name}")
                return ""
            return str(self.namespaces[ns][name])

        out = _RE.sub(repl, s)
        if return_missing:
            return out, missing
        if missing:
            raise InterpolatorError(f"Failed to interpolate: {', '.join(missing)}")
        return out

    def interpolate_or_error(self, s: str) -> str:
        return self.interpolate(s)


def interpolate_all(values: Dict[str, str], namespaces: Dict[str, Dict[str, str]]) -> Tuple[Dict[str, str], List[str]]:
    it = VariablesInterpolator(namespaces)
    out, missing = {}, []
    for k, v in values.items():
        r, m = it.interpolate(v, return_missing=True)
        out[k] = r
        missing += m
    return out, missing
