"""``${{ namespace.var }}`` interpolation (reference: ``utils/interpolator.py:19-84``).

Used for ``${{ secrets.NAME }}``, ``${{ env.NAME }}``, ``${{ run.args }}`` in configurations and
``${{ dstack.node_rank }}`` in volume names/paths.  ``$${{`` escapes a literal ``${{``.
"""

from __future__ import annotations

import re
from typing import Dict, List, Optional, Tuple

_NAME = re.compile(r"^([a-zA-Z_][a-zA-Z0-9_]*)\.([a-zA-Z_][a-zA-Z0-9_]*)$")


class InterpolatorError(ValueError):
    pass


class VariablesInterpolator:
    def __init__(self, namespaces: Dict[str, Dict[str, str]], skip: Optional[List[str]] = None):
        self.namespaces = namespaces
        self.skip = set(skip or [])

    def interpolate(self, s: str, return_missing: bool = False):
        """Single left-to-right scan: ``$${{`` -> literal ``${{``; ``${{ ns.name }}`` -> value;
        an unclosed pattern or an illegal name is an error (bash ``${VAR}`` is left alone)."""
        missing: List[str] = []
        out: List[str] = []
        i = 0
        while True:
            j = s.find("${{", i)
            if j < 0:
                out.append(s[i:])
                break
            if j > 0 and s[j - 1] == "$":  # escaped
                out.append(s[i:j - 1] + "${{")
                i = j + 3
                continue
            out.append(s[i:j])
            k = s.find("}}", j + 3)
            if k < 0:
                raise InterpolatorError(f"Unclosed pattern at position {j}: {s[j:j + 20]!r}")
            expr = s[j + 3:k].strip()
            m = _NAME.match(expr)
            if not m:
                raise InterpolatorError(f"Illegal reference name: {expr!r}")
            ns, name = m.group(1), m.group(2)
            i = k + 2
            if ns in self.skip:
                out.append(s[j:i])
                continue
            if ns not in self.namespaces:
                raise InterpolatorError(f"Unknown namespace `{ns}` in ${{{{ {expr} }}}}")
            if name not in self.namespaces[ns]:
                missing.append(f"{ns}.{name}")
                continue
            out.append(str(self.namespaces[ns][name]))
        res = "".join(out)
        if return_missing:
            return res, missing
        if missing:
            raise InterpolatorError(f"Failed to interpolate: {', '.join(missing)}")
        return res

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
