"""Import shim: exposes the package directory
``multi-modal-misinformation-detection-with-explanation-generation_amd/`` (whose name is
not a valid Python identifier) as the importable package ``mmf_amd``.

``import mmf_amd`` executes the package's ``__init__.py`` with ``__path__`` pointing at
that directory, so ``import mmf_amd.engine`` etc. resolve to files inside it.
"""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(
    os.path.dirname(os.path.abspath(__file__)),
    "multi-modal-misinformation-detection-with-explanation-generation_amd",
)

_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR]
)
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
