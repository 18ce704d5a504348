__all__ = ["groups"]
from .groups import LieGroupParameter, SO3, RxSO3, SE3, Sim3, cat, stack
