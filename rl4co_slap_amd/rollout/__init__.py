from .constructive import ConstructiveDecoder, ConstructivePolicy, LogitsDecoder, NoEncoder
from .engine import (CVRPFusedEpisode, CVRPStepwiseEpisode, SLAPFusedEpisode,
                     SLAPStepwiseEpisode, TSPFusedEpisode, TSPStepwiseEpisode)

__all__ = ["TSPStepwiseEpisode", "TSPFusedEpisode", "SLAPStepwiseEpisode", "SLAPFusedEpisode",
           "CVRPFusedEpisode", "CVRPStepwiseEpisode", "ConstructivePolicy",
           "ConstructiveDecoder", "LogitsDecoder", "NoEncoder"]
