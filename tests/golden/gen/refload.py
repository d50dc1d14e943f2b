"""Load the reference's hot-path modules from /root/reference (FIXTURE-GENERATION ONLY).

Runs only in the build container (the reference is absent on the GPU box).
Nothing is written under /root/reference: bytecode caching is disabled before
any reference module is imported.  The reference mixes top-level imports
(`from core.tracing import ...`) with package-relative ones that climb above the
top level (`from ..core import ...`), so the reference tree is imported as the
namespace package `reference` (parent dir on sys.path) and top-level names such
as `core` / `mathematics` are aliased onto `reference.core` / ... .
"""
import importlib
import importlib.abc
import importlib.util
import os
import sys

sys.dont_write_bytecode = True

REF_ROOT = "/root/reference"
_HERE = os.path.dirname(os.path.abspath(__file__))
_TOP = ("core", "mathematics", "accelerators", "io_utils", "debug")


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path=None, target=None):
        if fullname.split(".")[0] in _TOP:
            return importlib.util.spec_from_loader(fullname, self)
        return None

    def create_module(self, spec):
        mod = importlib.import_module("reference." + spec.name)
        return mod

    def exec_module(self, module):
        pass  # already executed under its `reference.` name


def install():
    if not os.path.isdir(REF_ROOT):
        raise RuntimeError("reference tree not present (fixture generation runs in the build container only)")
    sys.path.insert(0, os.path.join(_HERE, "standins"))
    parent = os.path.dirname(REF_ROOT)
    if parent not in sys.path:
        sys.path.insert(1, parent)
    if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _AliasFinder())
    import taichi  # noqa: F401  (the stand-in)
    return taichi
