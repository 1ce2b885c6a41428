"""Import alias for the ``audio-backdoor-attack_amd/`` package (its directory name is
not a Python identifier).  ``import abd_amd`` loads that directory as package
``abd_amd`` and replaces this shim in ``sys.modules``."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "audio-backdoor-attack_amd")
_spec = importlib.util.spec_from_file_location("abd_amd", os.path.join(_PKG_DIR, "__init__.py"),
                                               submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["abd_amd"] = _mod
_spec.loader.exec_module(_mod)
