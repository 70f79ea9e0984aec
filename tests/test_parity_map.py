"""The reference-suite parity map (``docs/reference/test-parity.yaml``) stays honest: every test it
names exists here, and -- where the reference checkout is present -- every reference server test
case is mapped (or marked ``n/a`` with a reason)."""

from __future__ import annotations

import importlib.util
from pathlib import Path

import pytest
import yaml

ROOT = Path(__file__).resolve().parents[1]


def _tool():
    spec = importlib.util.spec_from_file_location("test_parity_tool", ROOT / "tools/test_parity.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_every_mapped_test_exists():
    tool = _tool()
    mapping = yaml.safe_load((ROOT / "docs/reference/test-parity.yaml").read_text())
    ours = tool.our_tests()
    missing = []
    for f, cases in mapping.items():
        for case, target in cases.items():
            if isinstance(target, str) and target.startswith("n/a"):
                assert len(target) > 20, f"{f} {case}: n/a needs a reason"
                continue
            for t in (target if isinstance(target, list) else [target]):
                if t not in ours:
                    missing.append((f, case, t))
    assert not missing, missing


def test_every_reference_case_is_mapped():
    tool = _tool()
    if not tool.REF.is_dir():
        pytest.skip("reference checkout not present")
    mapping = yaml.safe_load((ROOT / "docs/reference/test-parity.yaml").read_text())
    unmapped = [(f, c) for f, cases in tool.reference_cases().items() for c in cases
                if c not in (mapping.get(f) or {})]
    assert not unmapped, unmapped
