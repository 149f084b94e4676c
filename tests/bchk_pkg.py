"""Load the product package (directory polar-codes-with-bch-kernel_amd/) as `bchk_amd`."""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "polar-codes-with-bch-kernel_amd")


def load():
    if "bchk_amd" in sys.modules:
        return sys.modules["bchk_amd"]
    spec = importlib.util.spec_from_file_location(
        "bchk_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["bchk_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
