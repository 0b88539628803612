import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def golden():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        return json.load(f)


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Which kernel-variant set the forced-variant tests ran on (tests/engines.py)."""
    try:
        from tests import engines
    except Exception:
        try:
            import engines  # tests/ on sys.path
        except Exception:
            return
    u = engines.USAGE
    if u["exp_lib"] is None and not u["exp_variant_runs"] and not u["skipped_variants"]:
        return
    terminalreporter.write_line(
        f"variant set: product library + experiments build {u['exp_lib'] or '(absent)'}; "
        f"{u['exp_variant_runs']} forced-variant switches to the experiments build; "
        f"skipped variants (SMOL_ALLOW_NO_EXP=1): {sorted(u['skipped_variants']) or 'none'}")
