"""
KeyFrame record (reference: slam_system/key_frame.py:13-107) — same fields and .mat export.

`feature_pts` holds keypoint objects with `.pt` (as cv2 returns) or an [N,2] array after
convert_keypoint_to_array(); `landmark_index` is the int32 global ray id of each feature.
"""
import numpy as np
import scipy.io as sio


def rotation_matrix_to_vector(R):
    """Rodrigues vector of a rotation matrix (stands in for cv.Rodrigues used at key_frame.py:97)."""
    R = np.asarray(R, np.float64)
    c = (np.trace(R) - 1.0) / 2.0
    c = min(1.0, max(-1.0, c))
    th = np.arccos(c)
    if th < 1e-12:
        return np.zeros(3)
    if np.pi - th < 1e-6:
        # axis from the symmetric part
        M = (R + np.eye(3)) / 2.0
        k = int(np.argmax(np.diag(M)))
        ax = M[:, k] / np.sqrt(M[k, k])
        return ax * th
    ax = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]) / (2.0 * np.sin(th))
    return ax * th


class KeyFrame:
    """A keyframe of the map (key_frame.py:16-51)."""

    def __init__(self, img, img_index, center, rotation, u, v, pan, tilt, f):
        self.img = img
        self.img_index = img_index
        self._lazy = None
        self._pts = np.ndarray(0)
        self._des = np.ndarray(0)
        self._lmi = []
        self.pan, self.tilt, self.f = pan, tilt, f
        self.center = center
        self.base_rotation = rotation
        self.u = u
        self.v = v

    # feature_pts / feature_des / landmark_index: plain attributes as in the reference; bundle_adjustment hands them
    # over as (all keypoints, all descriptors, a provider of the call's per-keyframe (local, global) lists in the
    # reference's set() order, this keyframe's position), and the lists are formed on first use -- a 30-keyframe
    # window re-creates every keyframe per BA call, and in a stream most are replaced before anything reads them
    def set_features_lazy(self, keypoints, descriptors, provider, position=None):
        """provider: an index array (this keyframe's selected features, no landmark ids) or an object whose
        lists(position) returns (local index array, global landmark id array)."""
        self._lazy = (keypoints, descriptors, provider, position)

    def _materialise(self):
        kps, des, prov, pos = self._lazy
        self._lazy = None
        if pos is None:
            idx = np.asarray(prov, np.int64)
        else:
            idx, glo = prov.lists(pos)
            self._lmi = glo.astype(np.int32)
        if isinstance(kps, np.ndarray):
            self._pts = np.asarray(kps)[idx]
        else:
            self._pts = list(map(kps.__getitem__, idx.tolist()))
        self._des = np.asarray(des).take(idx, axis=0)

    @property
    def landmark_index(self):
        if self._lazy is not None:
            self._materialise()
        return self._lmi

    @landmark_index.setter
    def landmark_index(self, value):
        if self._lazy is not None:
            self._materialise()
        self._lmi = value

    @property
    def feature_pts(self):
        if self._lazy is not None:
            self._materialise()
        return self._pts

    @feature_pts.setter
    def feature_pts(self, value):
        if self._lazy is not None:
            self._materialise()
        self._pts = value

    @property
    def feature_des(self):
        if self._lazy is not None:
            self._materialise()
        return self._des

    @feature_des.setter
    def feature_des(self, value):
        if self._lazy is not None:
            self._materialise()
        self._des = value

    def get_feature_num(self):
        if self._lazy is not None:
            self._materialise()
        return len(self._pts)

    def has_features(self):
        """get_feature_num() > 0, answered without forming the lists when they are still pending (a keyframe of a BA
        call has features iff it takes part in one of the call's matches)."""
        if self._lazy is not None and self._lazy[3] is not None:
            return self._lazy[2].nonempty(self._lazy[3])
        return self.get_feature_num() > 0

    def convert_keypoint_to_array(self, norm=True):
        """key_frame.py:59-73."""
        n = len(self.feature_pts)
        pts = np.zeros((n, 2), dtype=np.float64)
        for i in range(n):
            p = self.feature_pts[i]
            pts[i] = p.pt if hasattr(p, "pt") else p
        des = np.asarray(self.feature_des, dtype=np.float64)
        if norm and len(des):
            des = des / np.linalg.norm(des, axis=1).reshape(-1, 1)
        self.feature_pts = pts
        self.feature_des = des

    def save_to_mat(self, path):
        """key_frame.py:75-107: keys im_name, keypoint, descriptor, camera (9x1), ptz (3x1)."""
        if isinstance(self.feature_pts, list):
            self.convert_keypoint_to_array()
        br = np.asarray(self.base_rotation)
        save_br = rotation_matrix_to_vector(br) if br.shape == (3, 3) else br.ravel()
        data = {
            "im_name": str(self.img_index) + ".jpg",
            "keypoint": self.feature_pts,
            "descriptor": self.feature_des,
            "camera": np.array([self.u, self.v, self.f, save_br[0], save_br[1], save_br[2], self.center[0],
                                self.center[1], self.center[2]]).reshape(-1, 1),
            "ptz": np.array([self.pan, self.tilt, self.f]).reshape(-1, 1),
        }
        sio.savemat(path, mdict=data)
