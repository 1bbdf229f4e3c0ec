"""Engine objects (the flagship 'model' of this framework is the kNN engine)."""
from .knearests import KNearests

__all__ = ["KNearests"]
