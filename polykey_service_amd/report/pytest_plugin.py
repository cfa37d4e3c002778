"""pytest plugin: emit ``go test -json``-shaped events so the Jest reporter renders pytest runs.

The reference pipes ``go test -json`` into ``tparse`` / its beautifier (``Makefile:103-109``);
here ``pytest -p polykey_service_amd.report.pytest_plugin --jest-json=events.jsonl`` writes
``{"Action": "run"|"pass"|"fail"|"skip", "Package": <file>, "Test": <name>, "Elapsed": s}``
lines and ``python -m polykey_service_amd.report jest < events.jsonl`` prints the report
(``make test`` does both).
"""
from __future__ import annotations

import json


def pytest_addoption(parser):
    parser.addoption("--jest-json", default=None, help="write go-test-json style events to this file")


def pytest_configure(config):
    path = config.getoption("--jest-json")
    if path:
        config._jest_fh = open(path, "w")


def pytest_unconfigure(config):
    fh = getattr(config, "_jest_fh", None)
    if fh:
        fh.close()


def _emit(config, **ev):
    fh = getattr(config, "_jest_fh", None)
    if fh:
        fh.write(json.dumps(ev) + "\n")
        fh.flush()


def pytest_runtest_logstart(nodeid, location):
    pass


def pytest_runtest_logreport(report):
    import pytest
    config = pytest_runtest_logreport.config  # set in pytest_sessionstart
    pkg, _, test = report.nodeid.partition("::")
    if report.when == "setup" and report.passed:
        _emit(config, Action="run", Package=pkg, Test=test)
    if report.when == "setup" and report.skipped:
        _emit(config, Action="skip", Package=pkg, Test=test, Elapsed=0.0)
    elif report.when == "call":
        _emit(config, Action="pass" if report.passed else "fail", Package=pkg, Test=test,
              Elapsed=round(report.duration, 3))
    elif report.failed:
        _emit(config, Action="fail", Package=pkg, Test=test, Elapsed=round(report.duration, 3))


def pytest_sessionstart(session):
    pytest_runtest_logreport.config = session.config
