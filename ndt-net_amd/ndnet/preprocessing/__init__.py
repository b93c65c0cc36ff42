from .ndt_legacy import NDT_Sampler  # noqa: F401
from .ndtnet_preprocessing import ndt_preprocessing  # noqa: F401
