"""pytest configuration: the `gpu` marker and import paths.

The product package lives in `cuda-acceleratedvectordatabaseengine_amd/` (not a
Python identifier), so it is registered here as module `vdb_amd`. The oracle
(`oracle/`) is test infrastructure and is imported only by tests.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "cuda-acceleratedvectordatabaseengine_amd")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def load_vdb():
    if "vdb_amd" in sys.modules:
        return sys.modules["vdb_amd"]
    spec = importlib.util.spec_from_file_location("vdb_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vdb_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


load_vdb()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")
