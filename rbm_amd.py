"""Import shim for the product package.

The package directory is ``recommender-baseline-model_amd/`` (a name with
hyphens, so not importable by ``import``).  ``import rbm_amd`` executes this
file, which loads that directory as the package ``rbm_amd`` and replaces
itself in ``sys.modules``; ``import rbm_amd.models`` etc. then resolve inside
the directory.
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "recommender-baseline-model_amd")
_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_DIR, "__init__.py"),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
