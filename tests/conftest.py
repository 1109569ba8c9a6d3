import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"), os.path.join(REPO, "oracle"), REPO,
          os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: CPU test taking more than a few seconds")
    # The multi-process GPU test (test_gpu_multiprocess.py) starts its ranks from a forkserver, which
    # must exist before this process touches the GPU: its children are forked from a process that
    # never initialised HIP, and nothing is exec'ed from one that did. Started for every run (it is
    # cheap), whatever the -m expression: a plain `pytest tests` initialises HIP in earlier GPU tests,
    # and a forkserver started lazily after that would be a fork+exec from a GPU-initialised process.
    # The test skips unless RT_FORKSERVER_EARLY is set.
    import multiprocessing.forkserver
    multiprocessing.forkserver.ensure_running()
    os.environ["RT_FORKSERVER_EARLY"] = "1"


@pytest.fixture(scope="session")
def repo():
    return REPO


def pytest_collection_modifyitems(config, items):
    # A development variant of the library (scripts/build_variant.sh with -DRT_DEV_ONLY=n, selected by RT_HIP_LIB)
    # instantiates one kernel family and answers RT_ERR_UNSUPPORTED for the others -- the binary-BVH renders the
    # wide-tree tests compare against among them. Round 5 ran test_gpu_wide.py on such a variant and read its 8
    # refusals as wrong images; a GPU session on one now stops here instead.
    if not any(item.get_closest_marker("gpu") for item in items):
        return
    from rt_amd import abi
    info = abi.build_info()
    if info.get("dev_only", "0") != "0":
        pytest.exit(f"{abi.lib_path()} is a development build ({' '.join(f'{k}={v}' for k, v in info.items())}): "
                    "it renders one kernel family only; run the GPU tests on the full library", returncode=4)
