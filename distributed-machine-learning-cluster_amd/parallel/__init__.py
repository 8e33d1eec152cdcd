"""Parallelism: data-parallel inference over RCCL (native csrc/comm: scatter
u8 shards, gather top-1, elastic on GPU loss) and weight broadcast. The
reference's only parallelism is request-level data parallelism plus
splitting the cluster between two jobs; tensor/pipeline/
sequence/expert parallelism do not apply to a 224x224 CNN classifier served
at this size and are not provided."""
from .dp import DataParallelRunner, NodeGroup, broadcast_state_dict  # noqa: F401
