"""Import shim: ``import fedamw_amd`` loads the package directory
``non-iid-distributed-learning-with-optimal-mixture-weights_amd/`` (whose name is
not a Python identifier) under the importable name ``fedamw_amd``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                     'non-iid-distributed-learning-with-optimal-mixture-weights_amd')
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_DIR, '__init__.py'),
                                     submodule_search_locations=[_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
