"""User resource tags (``tags`` in the AWS/Azure/GCP backend configs), checked against each cloud's
rules when a backend is configured and merged into every resource the backend creates (reference
``C/backends/aws/resources.py:461-488``, ``azure/resources.py:78-100``, ``gcp/resources.py:327-353``).

The rules as each cloud documents them:

* AWS: key 1-128 and value 0-256 characters from letters, digits, space and ``_.:/=+-@``; keys may
  not start with ``aws:`` (reserved).
* Azure: key 1-512 characters without ``<>&\\%?/``; value up to 256 characters.
* GCP labels: key 1-63 characters, starting with a lowercase letter, then lowercase letters, digits,
  ``_`` and ``-``; value 0-63 of the same (no leading-letter rule).
"""

from __future__ import annotations

import re
from typing import Dict, Optional

from dstack_amd.core.errors import BackendError

_AWS = re.compile(r"[\w .:/=+\-@]*")
_AZURE_KEY_BAD = re.compile(r"[<>&\\%?/]")
_GCP_KEY = re.compile(r"[a-z][a-z0-9_\-]*")
_GCP_VALUE = re.compile(r"[a-z0-9_\-]*")


def aws_tag_key_ok(key: str) -> bool:
    return 1 <= len(key) <= 128 and not key.startswith("aws:") and _AWS.fullmatch(key) is not None


def aws_tag_value_ok(value: str) -> bool:
    return len(value) <= 256 and _AWS.fullmatch(value) is not None


def azure_tag_key_ok(key: str) -> bool:
    return 1 <= len(key) <= 512 and _AZURE_KEY_BAD.search(key) is None and "\n" not in key


def azure_tag_value_ok(value: str) -> bool:
    return len(value) <= 256 and "\n" not in value


def gcp_resource_name_ok(name: str) -> bool:
    """Also the rule for GCP resource names (instances, disks, firewalls)."""
    return 1 <= len(name) <= 63 and _GCP_KEY.fullmatch(name) is not None


def gcp_label_value_ok(value: str) -> bool:
    return len(value) <= 63 and _GCP_VALUE.fullmatch(value) is not None


_RULES = {
    "aws": (aws_tag_key_ok, aws_tag_value_ok, "Invalid resource tags",
            "AWS tag keys are 1-128 and values 0-256 characters of letters, digits, spaces and _.:/=+-@; "
            "keys may not start with 'aws:'"),
    "azure": (azure_tag_key_ok, azure_tag_value_ok, "Invalid Azure resource tags",
              "Azure tag keys are 1-512 characters without <>&\\%?/ and values at most 256"),
    "gcp": (gcp_resource_name_ok, gcp_label_value_ok, "Invalid resource labels",
            "GCP label keys start with a lowercase letter and, like values, hold at most 63 lowercase "
            "letters, digits, '_' and '-'"),
}


def validate_tags(cloud: str, tags: Optional[Dict[str, str]]) -> None:
    """Raise BackendError naming the offending keys when ``tags`` break ``cloud``'s rules."""
    if not tags:
        return None
    key_ok, value_ok, head, rule = _RULES[cloud]
    bad = [k for k, v in tags.items() if not (isinstance(k, str) and isinstance(v, str) and key_ok(k) and value_ok(v))]
    if bad:
        raise BackendError(f"{head}: {', '.join(map(repr, bad))}. {rule}")
    return None


def merged_tags(cloud: str, base: Dict[str, str], config: Optional[dict]) -> Dict[str, str]:
    """dstack's own tags (owner/project/...) plus the validated ``tags`` of the backend config; the
    user's win on a clash except for the ownership keys dstack relies on to find its resources."""
    user = (config or {}).get("tags") or {}
    validate_tags(cloud, user)
    return {**user, **base}
