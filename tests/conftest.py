import os
import sys

import pytest

try:  # import torch before the HIP library is loaded (see knn_amd.lib())
    import torch  # noqa: F401
except Exception:
    pass

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


def cout_double(x):
    """std::cout << double with default precision (6 significant, %g)."""
    return "%g" % x


@pytest.fixture(scope="session")
def fmt_cout():
    return cout_double


def pytest_terminal_summary(terminalreporter):
    """Exact-tie vote tally of the parity suite (test_gpu_parity.TIE_VOTES)."""
    mod = sys.modules.get("test_gpu_parity")
    tv = getattr(mod, "TIE_VOTES", None) if mod else None
    if not tv or not tv["cases"]:
        return
    terminalreporter.write_line(
        "tie-vote parity: %d cases, %d queries, %d with an exact-tie vote, %d of those with a "
        "label other than the oracle's std::sort order; %d re-ordered as the reference's "
        "std::sort" % (tv["cases"], tv["queries"], tv["tie_vote"], tv["tie_vote_label_differs"],
                       tv.get("reordered", 0)))
    try:
        import json
        out = os.path.join(ROOT, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "tie_votes.json"), "w") as f:
            json.dump(tv, f)
    except OSError:
        pass
