import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def pytest_runtest_logreport(report):
    """Print a failure's traceback the moment it happens: a GPU runtime abort later in the session (e.g. in a
    fixture teardown) would otherwise take the end-of-session summary with it."""
    if report.failed and os.environ.get("KAFKA_EAGER_FAILURES", "1") == "1":
        sys.stderr.write(f"\n==== FAILED {report.nodeid} ({report.when})\n{report.longreprtext}\n")
        sys.stderr.flush()
