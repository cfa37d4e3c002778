"""Test-only fault hooks, behind ONE explicit switch.

A fault hook makes a serving process deliberately wrong (a TP rank drops its attention partial,
a bench child hangs) so that a test can prove the surrounding checks catch it.  A stray
environment variable must never do that to a production server silently, so every hook is read
through :func:`get`: it is honoured only when ``POLYKEY_TEST_HOOKS=1`` is also set, and an active
hook is logged at ERROR on stderr (a set but ignored one at WARNING).
"""
from __future__ import annotations

import json
import os
import sys
from typing import Optional

SWITCH = "POLYKEY_TEST_HOOKS"


def enabled() -> bool:
    return os.environ.get(SWITCH) == "1"


def _log(level: str, msg: str, **kw) -> None:
    print(json.dumps({"level": level, "msg": msg, **kw}), file=sys.stderr, flush=True)


def get(name: str) -> Optional[str]:
    """The value of fault hook ``name`` when hooks are switched on, else None."""
    v = os.environ.get(name)
    if not v:
        return None
    if not enabled():
        _log("WARN", "test fault hook ignored (set POLYKEY_TEST_HOOKS=1 to enable it)", hook=name, value=v)
        return None
    _log("ERROR", "TEST FAULT HOOK ACTIVE: this process is deliberately faulty", hook=name, value=v)
    return v
