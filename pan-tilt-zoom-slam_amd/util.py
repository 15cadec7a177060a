"""
Host utilities on the BA / tracking path (reference: slam_system/util.py).

overlap_pan_angle (util.py:49-72) builds the BA pair mask and the keyframe trigger; get_overlap_index
(util.py:75-96) intersects observed and predicted ray indices in the EKF.  Both are O(N) host
bookkeeping, kept in Python as in the reference.  Plotting / dataset I/O helpers are out of scope.
"""
import math

import numpy as np
import scipy.io as sio


def overlap_pan_angle_half_fov(fl, im_width):
    """Half horizontal field of view (degrees) of a camera, as overlap_pan_angle forms it per camera."""
    return math.atan((im_width / 2) / fl) * 180.0 / math.pi


def overlap_pan_angle(fl_1, pan_1, fl_2, pan_2, im_width):
    """Overlapped pan angle (degrees) of two cameras, pan only, no wrap-around (util.py:49-72)."""
    d1 = overlap_pan_angle_half_fov(fl_1, im_width)
    d2 = overlap_pan_angle_half_fov(fl_2, im_width)
    return max(0, min(pan_1 + d1, pan_2 + d2) - max(pan_1 - d1, pan_2 - d2))


def get_overlap_index(index1, index2):
    """Positions of the shared values of two sorted arrays (util.py:75-96, same two-pointer merge)."""
    o1, o2 = [], []
    p1 = p2 = 0
    while p1 < len(index1) and p2 < len(index2):
        if index1[p1] == index2[p2]:
            o1.append(p1)
            o2.append(p2)
            p1 += 1
            p2 += 1
        elif index1[p1] < index2[p2]:
            p1 += 1
        else:
            p2 += 1
    return np.array(o1, dtype=np.int64), np.array(o2, dtype=np.int64)


def save_camera_pose(pan, tilt, zoom, path):
    """util.py:263-277: write pan/tilt/f lists to a .mat file."""
    sio.savemat(path, mdict={"pan": np.asarray(pan), "tilt": np.asarray(tilt), "f": np.asarray(zoom)})


def load_camera_pose(path, separate=False):
    """util.py:280-298."""
    d = sio.loadmat(path)
    pan, tilt, f = d["pan"].squeeze(), d["tilt"].squeeze(), d["f"].squeeze()
    if separate:
        return pan, tilt, f
    return np.stack([pan, tilt, f], 1)
