"""Register the package directory `puffer-phc_amd/` under the importable name `puffer_phc_amd`.

The directory name carries a hyphen (repository convention), which Python cannot import
directly; this helper loads its `__init__.py` with the right submodule search path.
"""

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "puffer-phc_amd")


def register():
    if "puffer_phc_amd" in sys.modules:
        return sys.modules["puffer_phc_amd"]
    spec = importlib.util.spec_from_file_location(
        "puffer_phc_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR]
    )
    mod = importlib.util.module_from_spec(spec)
    sys.modules["puffer_phc_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
