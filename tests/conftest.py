import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "sat-mpi-stana-andrei_amd")
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


def clause_set_sha(clauses):
    """sha256 of a clause SET in make_golden_bench.py's canonical form (each
    clause sorted, the clauses sorted, compact JSON)."""
    import hashlib
    import json
    s = json.dumps(sorted(sorted(c) for c in clauses), separators=(",", ":"))
    return hashlib.sha256(s.encode()).hexdigest()


def clause_list_sha(clauses):
    """sha256 of an ORDERED clause list (clause and literal order kept)."""
    import hashlib
    import json
    s = json.dumps([list(c) for c in clauses], separators=(",", ":"))
    return hashlib.sha256(s.encode()).hexdigest()
