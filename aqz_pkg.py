"""Import helper: the package directory is `acquire-zarr_amd/` (hyphenated),
so it is registered in sys.modules as `acquire_zarr_amd` from its path."""
from __future__ import annotations

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "acquire-zarr_amd")


def load():
    mod = sys.modules.get("acquire_zarr_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "acquire_zarr_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["acquire_zarr_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
