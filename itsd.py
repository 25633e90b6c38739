"""Import shim: exposes the package directory
``inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd/``
(whose name is not a valid Python identifier) as the importable package ``itsd``.

``import itsd`` executes this file once; it loads the real package under the same
name and replaces itself in ``sys.modules``, so ``from itsd.search import
RandomSearch`` etc. resolve to the package's submodules.
"""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(
    os.path.dirname(os.path.abspath(__file__)),
    "inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd",
)

_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR]
)
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
