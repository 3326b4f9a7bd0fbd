"""Import shim: the package lives in the directory ``joss-nifty_amd/`` (not a
valid Python identifier); ``import nifty_amd`` loads it under this name."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_pkg_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "joss-nifty_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_pkg_dir, "__init__.py"),
                                     submodule_search_locations=[_pkg_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
