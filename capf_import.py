"""Import helper: exposes the `cypher-for-apache-flink_amd/` package as `capf_amd`."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "cypher-for-apache-flink_amd")


def load():
    if "capf_amd" in sys.modules:
        return sys.modules["capf_amd"]
    spec = importlib.util.spec_from_file_location(
        "capf_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["capf_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


load()
