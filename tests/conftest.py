import faulthandler
import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"


HANG_DUMP_S = 100     # below pytest's 120 s per-test limit (pytest.ini) and gpurun's 180 s silence kill
_dump_file = None


def pytest_configure(config):
    global _dump_file
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmk.so on cuda:0)")
    # Stalls must name where they are: a test still running after HANG_DUMP_S dumps every Python
    # thread's stack from faulthandler's own C thread (no GIL needed) into gpurun_out/, which
    # survives a killed GPU call.  The suite runs the library's shipped launch pattern: libmk's stall
    # watchdog (a progress dispatch after every launch) stays off unless MK_WATCHDOG is set by the
    # caller (e.g. MK_WATCHDOG=60 when chasing a stall; it then logs to gpurun_out/watchdog.log).
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    if os.environ.get("MK_WATCHDOG"):
        os.environ.setdefault("MK_WATCHDOG_LOG", os.path.join(out, "watchdog.log"))
    _dump_file = open(os.path.join(out, "hang_dump.log"), "a")


def pytest_collection_modifyitems(config, items):
    # pytest.ini's 120 s limit is for the GPU tests (below gpurun's silence kill); the CPU tests that
    # run oracle chains get more room on a loaded host
    for item in items:
        if item.get_closest_marker("gpu") is None and item.get_closest_marker("timeout") is None:
            item.add_marker(pytest.mark.timeout(900))


@pytest.fixture(autouse=True)
def _dump_stacks_if_hung(request):
    if _dump_file is not None:
        _dump_file.write(f"--- {request.node.nodeid}\n")
        _dump_file.flush()
        faulthandler.dump_traceback_later(HANG_DUMP_S, exit=False, file=_dump_file)
    yield
    faulthandler.cancel_dump_traceback_later()


@pytest.fixture(scope="session")
def mk():
    return importlib.import_module(PKG)

