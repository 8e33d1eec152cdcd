"""Import alias for the framework package.

The framework lives in ``distributed-machine-learning-cluster_amd/`` (the
directory name required by the project layout is not a valid Python
identifier), so ``import dmlc`` maps onto that directory: every submodule
(``dmlc.models``, ``dmlc.ops``, ``dmlc.parallel``, ``dmlc.utils``, ...) is
resolved from there.
"""
import os as _os

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                         "distributed-machine-learning-cluster_amd")
__path__ = [_PKG_DIR]  # noqa: F821  (package path redirection)
_init = _os.path.join(_PKG_DIR, "__init__.py")
with open(_init) as _f:
    exec(compile(_f.read(), _init, "exec"))
