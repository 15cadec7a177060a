"""
Map of keyframes and global ray landmarks (reference: slam_system/scene_map.py:18-168).

`Map.add_keyframe_with_ba` re-runs bundle adjustment over all keyframes, as the reference does
(scene_map.py:53-117), on the GPU.  `RandomForestMap` keeps the reference's sliding-window BA
(`bundle_adjustment_processing`, last `max_ba_frame` keyframes, scene_map.py:198-244); its random-forest
relocaliser (C++ rf_map via ctypes) is out of scope and raises if used.

Both keep a correspondence.CorrespondenceCache keyed by KeyFrame.img_index: the reference re-detects
every keyframe and re-matches every pair on each BA call; here only the new keyframe is detected and
only its pairs are matched, with identical results.
"""
import time

import numpy as np
import scipy.io as sio

from bundle_adjustment import bundle_adjustment
from correspondence import CorrespondenceCache
from key_frame import KeyFrame
from util import overlap_pan_angle


class Map:
    """max_ba_frame: None (the reference: every keyframe is adjusted) or N: only the last N keyframes are
    adjusted, older ones stay as they are (RandomForestMap's window rule, scene_map.py:198-244; the
    streaming config's 30-keyframe window)."""

    def __init__(self, feature_method, cache_correspondences=True, max_ba_frame=None):
        assert feature_method in ("sift", "orb", "latch")
        self.global_ray = np.ndarray([0, 2])
        self.keyframe_list = []
        self.feature_method = feature_method
        self.ba_options = {}
        self.last_ba_time = None
        self.max_ba_frame = max_ba_frame
        self.correspondences = CorrespondenceCache() if cache_correspondences else None

    def add_first_keyframe(self, keyframe, verbose=False):
        assert isinstance(keyframe, KeyFrame)
        self.keyframe_list = [keyframe]
        if self.correspondences is not None and getattr(keyframe, "img", None) is not None:
            self.correspondences.prepare(keyframe.img_index, keyframe.img, self.feature_method)
        if verbose:
            print("first key frame is added, no bundle adjustment and landmark")

    def add_keyframe_without_ba(self, keyframe, verbose=False):
        assert isinstance(keyframe, KeyFrame)
        self.keyframe_list.append(keyframe)

    def add_keyframe_with_ba(self, keyframe, save_path, verbose=False):
        """scene_map.py:53-117: append, BA over all keyframes, keep keyframes with features."""
        assert isinstance(keyframe, KeyFrame)
        assert len(self.keyframe_list) >= 1
        ref = self.keyframe_list[0]
        self.add_keyframe_without_ba(keyframe, False)
        kept = []
        if self.max_ba_frame and len(self.keyframe_list) > self.max_ba_frame:
            kept = self.keyframe_list[:-self.max_ba_frame]
            self.keyframe_list = self.keyframe_list[-self.max_ba_frame:]
            if self.correspondences is not None:
                self.correspondences.retain([k.img_index for k in self.keyframe_list])
        n = len(self.keyframe_list)
        images = [k.img for k in self.keyframe_list]
        image_indices = [k.img_index for k in self.keyframe_list]
        initial_ptzs = np.array([[k.pan, k.tilt, k.f] for k in self.keyframe_list], dtype=np.float64).reshape(n, 3)
        start = time.time()
        landmarks, keyframes = bundle_adjustment(images, image_indices, self.feature_method, initial_ptzs, ref.center,
                                                 ref.base_rotation, ref.u, ref.v, save_path, verbose,
                                                 correspondences=self.correspondences, **self.ba_options)
        end = time.time()
        self.keyframe_list.pop()
        self.global_ray = landmarks
        self.keyframe_list = list(kept)
        for i, kf in enumerate(keyframes):
            if kf.has_features():  # (get_feature_num() > 0 without forming the lists: they are formed on first use)
                self.keyframe_list.append(kf)
            else:
                print("warning: key frame, %d, image index %d is not included in the map" % (i, image_indices[i]))
        if verbose:
            print("updated map, number of key frame: %d, number of landmark %d" % (len(self.keyframe_list),
                                                                                 len(landmarks)))
        self.last_ba_time = end - start
        print("BA time", end - start)
        return landmarks, self.keyframe_list

    def good_new_keyframe(self, ptz, threshold1=5, threshold2=20, im_width=1280, verbose=False):
        """scene_map.py:119-149: max pan overlap with existing keyframes in (threshold1, threshold2)."""
        ptz = np.asarray(ptz)
        assert ptz.shape[0] == 3
        if len(self.keyframe_list) == 0:
            print("Warning: not existing key frames")
            return False
        ov = [overlap_pan_angle(ptz[2], ptz[0], k.f, k.pan, im_width) for k in self.keyframe_list]
        if verbose:
            print("candidate key frame overlap: ", ov)
        m = max(ov)
        return threshold1 < m < threshold2

    def save_keyframes_to_mat(self, path):
        kfs = [{"index": k.img_index, "ptz": np.array([k.pan, k.tilt, k.f]), "center": k.center,
                "base_rotation": k.base_rotation, "principal_point": np.array([k.u, k.v])} for k in self.keyframe_list]
        sio.savemat(path, mdict={"keyframes": kfs})


class RandomForestMap:
    """Sliding-window BA of scene_map.py:171-244: the last `max_ba_frame` keyframes are adjusted (the first
    of them is the gauge, bundle_adjustment fixes frame 0), older keyframes are kept as they are.  The
    random-forest map files / relocaliser (rf_map, C++) are not part of this build."""

    def __init__(self, max_ba_frame=10, feature_method="sift", cache_correspondences=True):
        self.keyframe_list = []
        self.feature_method = feature_method
        self.max_ba_frame = max_ba_frame
        self.global_ray = np.ndarray([0, 2])
        self.ba_options = {}
        self.correspondences = CorrespondenceCache() if cache_correspondences else None

    def add_keyframe(self, keyframe):
        self.keyframe_list.append(keyframe)
        if len(self.keyframe_list) > 1:
            self.bundle_adjustment_processing()

    def bundle_adjustment_processing(self, save_path="./bundle_result", verbose=False):
        ref = self.keyframe_list[0]
        n = len(self.keyframe_list)
        window = [k for i, k in enumerate(self.keyframe_list) if i >= n - self.max_ba_frame]
        kept = [k for i, k in enumerate(self.keyframe_list) if i < n - self.max_ba_frame]
        images = [k.img for k in window]
        idx = [k.img_index for k in window]
        ptzs = np.array([[k.pan, k.tilt, k.f] for k in window], dtype=np.float64)
        if self.correspondences is not None:
            self.correspondences.retain(idx)
        landmarks, kfs = bundle_adjustment(images, idx, self.feature_method, ptzs, ref.center, ref.base_rotation, ref.u,
                                           ref.v, save_path, verbose, correspondences=self.correspondences,
                                           **self.ba_options)
        self.global_ray = landmarks  # window-local ray ids (the reference discards them)
        self.keyframe_list = kept
        for i, kf in enumerate(kfs):
            if kf.get_feature_num() > 0:
                kf.convert_keypoint_to_array()
                self.keyframe_list.append(kf)
            else:
                print("warning: key frame, %d, image index %d is not included in the map" % (i, idx[i]))
        return landmarks, kfs

    def relocalize(self, keyframe, ptz):
        raise NotImplementedError("random-forest relocalisation (C++ rf_map) is out of scope for this build")
