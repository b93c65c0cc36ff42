"""TEST INFRASTRUCTURE ONLY (the checker, never the product): a restatement of
the reference's CARLA_Seg.get_data_pcl (ndnet/datasets/CARLA_Seg.py:97-175)
in plain Python, for the parity tests of the native PLY reader and of
ndnet.datasets.CARLA_Seg.  Parity pinned by construction: the reference's own
loop (readlines, strip().split(), float() of tokens 0-2, int() of the last
token, the class bound, np.random.choice without replacement, float32 points,
one-hot of n_classes + 1), minus open3d (imported but unused on that path).
"""
import numpy as np


def get_data_pcl(pcl_filename, n_classes, n_samples, num_header_lines=10):
    points, classes = [], []
    with open(pcl_filename, "r") as f:
        pcl = f.readlines()                                    # CARLA_Seg.py:113-115
    for point in pcl[num_header_lines:]:                       # :118
        data = point.strip().split()                           # :120
        x, y, z = float(data[0]), float(data[1]), float(data[2])
        class_tag = int(data[-1])                              # :124
        if class_tag > n_classes:                              # :126-127
            raise ValueError(f"Class tag {class_tag} out of bounds")
        points.append(np.array([x, y, z]))
        classes.append(class_tag)
    np_points = np.asarray(points)
    point_indexes = np.random.choice(np_points.shape[0], n_samples, replace=False)  # :137-138
    np_points = np_points[point_indexes]
    np_classes = np.asarray(classes, dtype=np.uint16)[point_indexes]                # :142-143
    pts = np_points.astype(np.float32)                                              # :164 torch.tensor(...).float()
    gt = np.zeros((np_classes.shape[0], n_classes + 1), np.float32)                 # :167-170
    for i in range(np_classes.shape[0]):
        gt[i, int(np_classes[i])] = 1
    return pts, gt
