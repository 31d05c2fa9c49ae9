"""Small helpers used by the e2e drivers and logs
(reference ``pkg/util/util.go:29-74``: ``Pformat``, ``RandString``)."""
from __future__ import annotations

import json
import secrets

_ALPHABET = "0123456789abcdefghijklmnopqrstuvwxyz"


def pformat(value) -> str:
    """Pretty JSON for logs; strings pass through; unserialisable -> repr."""
    if isinstance(value, str):
        return value
    try:
        return json.dumps(value, indent=2, sort_keys=False, default=str)
    except (TypeError, ValueError):
        return repr(value)


def rand_string(n: int) -> str:
    """Random lowercase-alphanumeric string (a valid DNS-1035 label body)."""
    return "".join(secrets.choice(_ALPHABET) for _ in range(n))
