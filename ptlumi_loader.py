"""Import shim for the package directory ``path-tracing...but-on-the-lumi-cluster_amd``.

That directory name is not a valid Python identifier, so it is registered in
``sys.modules`` as ``ptlumi``; afterwards ``import ptlumi`` and
``from ptlumi import native`` work normally.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "path-tracing...but-on-the-lumi-cluster_amd")
NAME = "ptlumi"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod


load()
