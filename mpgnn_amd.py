"""Import shim: ``import mpgnn_amd`` loads the package in ./mpgnn-metapath-graph-neural-network_amd/
(the required directory name contains hyphens, which Python cannot import directly)."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "mpgnn-metapath-graph-neural-network_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
