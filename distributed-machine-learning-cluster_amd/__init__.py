"""dmlc — an MI355X-native distributed batch-inference cluster.

Same capabilities as tonychang04/distributed-machine-learning-cluster (ring
heartbeat membership, replicated versioned SDFS, two concurrent predict jobs
with fair share, leader fail-over with job resume, ``jobs`` percentile
reports, libtorch ``.ot`` checkpoints), rebuilt around:

* hand-written CDNA4 HIP kernels (``csrc/kernels``) for the CNN forward,
* a C++ engine with HBM-resident folded weights and hipGraph replay,
* RCCL (``torch.distributed`` backend "nccl") scatter/gather over xGMI for
  data-parallel inference across the GPUs of a node,
* a C++17 control plane (``csrc/control``, ``csrc/serve``, ``csrc/cli``).

Import as ``import dmlc``.
"""
__version__ = "0.1.0"

import os as _os

PACKAGE_DIR = _os.path.abspath(__path__[0])  # noqa: F821  (set by the dmlc import alias)
REPO_ROOT = _os.path.dirname(PACKAGE_DIR)


def native():
    """Return the native extension module, loading torch first so that the
    HIP runtime shared by torch and the extension is initialised once."""
    import importlib
    import torch  # noqa: F401
    return importlib.import_module(__name__ + "._C")
