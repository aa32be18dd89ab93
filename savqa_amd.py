"""Import shim: the package lives in ./structured-alignment-vqa_amd/ (a directory name
that is not a Python identifier); `import savqa_amd` loads it from there."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "structured-alignment-vqa_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_DIR, "__init__.py"),
                                     submodule_search_locations=[_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
