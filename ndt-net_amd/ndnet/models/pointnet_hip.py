"""HIP forward of NDTNetSegmentation (eval mode): placeholder until the MFMA kernels land."""


def available() -> bool:
    return False


def segmentation_forward(model, points, covariances):
    raise RuntimeError("HIP PointNet forward not built")
