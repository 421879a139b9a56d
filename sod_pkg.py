"""Import helper for the product package.

The package directory is ``sift-based-od_amd/`` (the layout the build contract
names); a hyphenated directory is not importable with a plain ``import``, so
this helper registers it under the module name ``sift_based_od_amd``::

    import sod_pkg
    sod = sod_pkg.load()          # == import sift_based_od_amd
    from sift_based_od_amd import synthetic
"""
import importlib.util
import os
import sys

NAME = "sift_based_od_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sift-based-od_amd")


def load():
    mod = sys.modules.get(NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(NAME, None)
        raise
    return mod
