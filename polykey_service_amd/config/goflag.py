"""A local (non-global) Go ``flag``-package compatible parser.

The reference registers ``-server -timeout -log-level -env`` on Go's *global* FlagSet and
calls ``flag.Parse()`` (``internal/config/config.go:177-183``); a second ``Load()`` there
panics with "flag redefined" (SURVEY.md §2.5 #12).  This parser is instantiated per call
and accepts Go's syntax: ``-name value``, ``-name=value``, ``--name=value``, bare
``-boolflag``; parsing stops at the first non-flag argument or at ``--``.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple


class FlagError(ValueError):
    pass


class FlagSet:
    def __init__(self, name: str = "polykey"):
        self.name = name
        self._defs: Dict[str, Tuple[Callable[[str], object], object, str, bool]] = {}
        self.values: Dict[str, object] = {}
        self.args: List[str] = []
        self.seen: set = set()

    def _define(self, name: str, conv, default, usage: str, is_bool: bool = False) -> None:
        if name in self._defs:
            raise FlagError(f"{self.name} flag redefined: {name}")
        self._defs[name] = (conv, default, usage, is_bool)
        self.values[name] = default

    def string(self, name: str, default: str = "", usage: str = "") -> None:
        self._define(name, str, default, usage)

    def duration(self, name: str, default: float = 0.0, usage: str = "") -> None:
        from ..utils.slog import parse_go_duration
        self._define(name, parse_go_duration, default, usage)

    def int(self, name: str, default: int = 0, usage: str = "") -> None:
        self._define(name, lambda s: int(s, 0), default, usage)

    def float(self, name: str, default: float = 0.0, usage: str = "") -> None:
        self._define(name, float, default, usage)

    def bool(self, name: str, default: bool = False, usage: str = "") -> None:
        def conv(s: str) -> bool:
            low = s.lower()
            if low in ("1", "t", "true"):
                return True
            if low in ("0", "f", "false"):
                return False
            raise FlagError(f"invalid boolean value {s!r}")
        self._define(name, conv, default, usage, is_bool=True)

    def parse(self, argv: Sequence[str]) -> "FlagSet":
        i, argv = 0, list(argv)
        while i < len(argv):
            a = argv[i]
            if len(a) < 2 or a[0] != "-":
                break
            if a == "--":
                i += 1
                break
            name = a[2:] if a.startswith("--") else a[1:]
            if not name or name[0] in "-=":
                raise FlagError(f"bad flag syntax: {a}")
            value: Optional[str] = None
            if "=" in name:
                name, value = name.split("=", 1)
            if name not in self._defs:
                raise FlagError(f"flag provided but not defined: -{name}")
            conv, _, _, is_bool = self._defs[name]
            if value is None:
                if is_bool:
                    value = "true"
                else:
                    if i + 1 >= len(argv):
                        raise FlagError(f"flag needs an argument: -{name}")
                    i += 1
                    value = argv[i]
            try:
                self.values[name] = conv(value)
            except (ValueError, FlagError) as e:
                raise FlagError(f"invalid value {value!r} for flag -{name}: {e}") from None
            self.seen.add(name)
            i += 1
        self.args = argv[i:]
        return self

    def usage(self) -> str:
        lines = [f"Usage of {self.name}:"]
        for n, (_, d, u, b) in self._defs.items():
            lines.append(f"  -{n}{'' if b else ' value'}\n    \t{u} (default {d!r})")
        return "\n".join(lines)

    def __getitem__(self, name: str):
        return self.values[name]
