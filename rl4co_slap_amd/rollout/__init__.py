from .engine import SLAPFusedEpisode, SLAPStepwiseEpisode, TSPFusedEpisode, TSPStepwiseEpisode

__all__ = ["TSPStepwiseEpisode", "TSPFusedEpisode", "SLAPStepwiseEpisode", "SLAPFusedEpisode"]
