// PointNet (NDTNetSegmentation) forward kernels: see pointnet_kernels.hip.
#pragma once
