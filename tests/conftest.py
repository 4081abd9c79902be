import importlib.util
import os
import sys

import pytest

# every streaming context of the GPU suite verifies its arena's guard gaps at each batch sync (a
# kernel writing past one of its buffers fails the test with the buffer's index instead of
# corrupting a neighbour silently); read once, when the library allocates its first arena buffer
os.environ.setdefault("PQH_ARENA_CHECK", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP path)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_package():
    """Import the product package from the `parquet-go_amd/` directory as `parquet_go_amd`."""
    name = "parquet_go_amd"
    if name in sys.modules:
        return sys.modules[name]
    pkg_dir = os.path.join(ROOT, "parquet-go_amd")
    spec = importlib.util.spec_from_file_location(name, os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def pq():
    return load_package()


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as o

    o.lib()
    return o
