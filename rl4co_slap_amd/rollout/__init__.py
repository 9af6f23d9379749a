from .engine import SLAPStepwiseEpisode, TSPFusedEpisode, TSPStepwiseEpisode

__all__ = ["TSPStepwiseEpisode", "TSPFusedEpisode", "SLAPStepwiseEpisode"]
