"""UNIVERSE / UNIVERSE++ networks (MI355X engine behind the reference API)."""
from .condition import ConditionerNetwork
from .score import ScoreNetwork
from .universe import Universe, UniverseGAN

__all__ = ["Universe", "UniverseGAN", "ScoreNetwork", "ConditionerNetwork"]
