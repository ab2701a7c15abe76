"""Loads the ``stl.fusion_amd`` package (its directory name contains a dot) as ``stl_fusion_amd``."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "stl.fusion_amd")


def load():
    mod = sys.modules.get("stl_fusion_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location("stl_fusion_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["stl_fusion_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
