from .engine import SLAPStepwiseEpisode, TSPStepwiseEpisode

__all__ = ["TSPStepwiseEpisode", "SLAPStepwiseEpisode"]
