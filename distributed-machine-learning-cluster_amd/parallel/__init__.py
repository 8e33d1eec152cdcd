"""Parallelism: data-parallel inference over RCCL (scatter u8 shards, gather
top-1), weight broadcast. The reference's only parallelism is request-level
data parallelism plus splitting the cluster between two jobs (SURVEY.md
§2.3); tensor/pipeline/sequence/expert parallelism do not apply to a
224x224 CNN classifier served at this size and are not provided."""
from .dp import DPInference, broadcast_state_dict  # noqa: F401
from .elastic import ElasticDPInference, RankLost  # noqa: F401
