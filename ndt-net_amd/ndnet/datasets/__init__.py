from .carla_seg import CARLA_Seg  # noqa: F401
