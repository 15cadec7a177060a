"""
PtzSlam (reference: slam_system/ptz_slam.py:21-539) — same attributes, methods and call order.

The per-frame hot part — projection of every ray, the FD measurement Jacobian, the Kalman update of
pose, rays and the dense state covariance, ray removal/addition — runs in libptzba (ptzekf_*): the
rays and the covariance live in device memory between frames (EKFHandle).  `rays` and `state_cov`
remain readable/assignable attributes as in the reference: reading returns a host copy of the device
state, assigning uploads it before the next device operation (in-place edits of a returned copy are
not written back).

The front-end (SIFT detection, LK flow + homography RANSAC) is reached through image_process hooks,
and relocalisation through relocalization.py / RandomForestMap, as in the reference.
"""
import copy

import numpy as np

import ptzba
from image_process import detect_compute_sift_array, keypoints_masking, matching_and_ransac
from key_frame import KeyFrame
from scene_map import Map, RandomForestMap


class PtzSlam:
    def __init__(self):
        # global rays and covariance matrix (device-resident once the tracker starts, see _ekf)
        self._rays = np.ndarray([0, 2])
        self._cov = np.zeros([3, 3])
        self._dirty = True  # host copies newer than the device state
        self._ekf = None

        self.previous_img = None
        self.previous_keypoints = None
        self.previous_keypoints_index = None
        self.des = np.ndarray([0, 128])
        self.current_camera = None
        self.keyframe_map = Map('sift')
        self.rf_map = RandomForestMap()
        self.cameras = []
        self.velocity = np.zeros(3)
        self.new_keyframe = False
        self.tracking_lost = False
        self.bad_tracking_cnt = 0
        self.keypoint_num = 500
        self.observe_var = 0.1
        self.angle_var = 0.001
        self.f_var = 1
        self.device = ptzba.default_device()

    # ------------------------------------------------------------------ device-backed state
    @property
    def rays(self):
        if self._dirty or self._ekf is None:
            return self._rays
        return self._ekf.get_state(rays=True, cov=False)[0]

    @rays.setter
    def rays(self, value):
        self._pull()
        self._rays = np.asarray(value, dtype=np.float64).reshape(-1, 2)
        self._dirty = True

    @property
    def state_cov(self):
        if self._dirty or self._ekf is None:
            return self._cov
        return self._ekf.get_state(rays=False, cov=True)[1]

    @state_cov.setter
    def state_cov(self, value):
        self._pull()
        self._cov = np.asarray(value, dtype=np.float64)
        self._dirty = True

    def _pull(self):
        if not self._dirty and self._ekf is not None:
            self._rays, self._cov = self._ekf.get_state()
            self._dirty = True

    def _push(self):
        if self._ekf is None:
            self._ekf = ptzba.EKFHandle(self.device)
        if self._dirty:
            self._ekf.set_state(self._rays, self._cov)
            self._dirty = False
        return self._ekf

    @staticmethod
    def _disp(camera):
        d = getattr(camera, "displacement", None)
        return None if d is None or not np.any(np.asarray(d) != 0) else np.asarray(d, np.float64)

    # ------------------------------------------------------------------ ptz_slam.py:73-138
    def compute_h_jacobian(self, pan, tilt, focal_length, rays):
        """Dense H [2R, 3+2R] of h(x) by the reference's central differences (0.001 deg, 0.1 px),
        with the intrinsics / displacement of the first camera (ptz_slam.py:92)."""
        cam = self.cameras[0]
        return ptzba.h_jacobian(cam.principal_point[0], cam.principal_point[1], focal_length, pan, tilt,
                                np.asarray(rays, np.float64).reshape(-1, 2), self._disp(cam), device=self.device)

    # ------------------------------------------------------------------ ptz_slam.py:140-208
    def init_system(self, img, camera, bounding_box=None):
        first_img_kp, first_des = detect_compute_sift_array(img, self.keypoint_num)
        if bounding_box is not None:
            masked_index = keypoints_masking(first_img_kp, bounding_box)
            first_img_kp = first_img_kp[masked_index]
            first_des = first_des[masked_index]
        init_rays = camera.back_project_to_rays(first_img_kp)
        self._rays = np.asarray(init_rays, np.float64).reshape(-1, 2).copy()
        self.des = first_des
        cov = self.angle_var * np.eye(3 + 2 * len(self._rays))
        cov[2][2] = self.f_var
        self._cov = cov
        self._dirty = True
        self._push()
        self.previous_img = img
        self.previous_keypoints = first_img_kp
        self.previous_keypoints_index = np.array([i for i in range(len(self._rays))])
        self.cameras.append(camera)

    # ------------------------------------------------------------------ ptz_slam.py:210-289
    def ekf_update(self, observed_keypoints, observed_keypoint_index, height, width):
        ekf = self._push()
        cam = self.current_camera
        ptz, vel, _ = ekf.update(cam.principal_point[0], cam.principal_point[1],
                                 [cam.pan, cam.tilt, cam.focal_length], observed_keypoints, observed_keypoint_index,
                                 height, width, self.observe_var, self._disp(cam))
        # the reference adds K y to the attributes directly (no matrix recompute), ptz_slam.py:265-268
        cam.pan, cam.tilt, cam.focal_length = float(ptz[0]), float(ptz[1]), float(ptz[2])
        self.current_camera = cam
        self.velocity = vel

    # ------------------------------------------------------------------ ptz_slam.py:291-315
    def remove_rays(self, index):
        delete_index = np.asarray(index).reshape(-1).astype(np.int64)
        if len(delete_index) == 0:
            return
        ekf = self._push()
        self.des = np.delete(self.des, delete_index, axis=0)
        ekf.remove_rays(delete_index)

    # ------------------------------------------------------------------ ptz_slam.py:317-388
    def add_rays(self, img, bounding_box):
        height, width = img.shape[0:2]
        ekf = self._push()
        cam = self.current_camera
        keypoints, keypoints_index = ekf.project_visible(cam.principal_point[0], cam.principal_point[1],
                                                         [cam.pan, cam.tilt, cam.focal_length], height, width,
                                                         self._disp(cam))
        new_keypoints, new_des = detect_compute_sift_array(img, self.keypoint_num)
        if bounding_box is not None:
            bounding_box_mask_index = keypoints_masking(new_keypoints, bounding_box)
            new_keypoints = new_keypoints[bounding_box_mask_index]
            new_des = new_des[bounding_box_mask_index]

        # remove keypoints within 50 px of the projected existing rays (ptz_slam.py:357-370): the reference zeroes
        # a 100 x 100 box of a mask per existing point, then keeps the keypoints whose integer pixel is still 1;
        # the same boxes (same integer bounds) tested against all keypoints at once
        kp_old = np.asarray(keypoints, np.float64).reshape(-1, 2)
        nk = np.asarray(new_keypoints, np.float64).reshape(-1, 2)
        if len(kp_old) and len(nk):
            ylo = np.maximum(0.0, kp_old[:, 1] - 50).astype(np.int64)
            yhi = np.minimum(float(height), kp_old[:, 1] + 50).astype(np.int64)
            xlo = np.maximum(0.0, kp_old[:, 0] - 50).astype(np.int64)
            xhi = np.minimum(float(width), kp_old[:, 0] + 50).astype(np.int64)
            xi, yi = nk[:, 0].astype(np.int64), nk[:, 1].astype(np.int64)
            covered = np.zeros(len(nk), bool)
            for a in range(0, len(kp_old), 256):  # bounded temporaries
                b = slice(a, a + 256)
                covered |= ((ylo[b, None] <= yi) & (yi < yhi[b, None]) & (xlo[b, None] <= xi) & (xi < xhi[b, None])).any(0)
            existing_keypoints_mask_index = np.flatnonzero(~covered).astype(np.int32)
        else:
            existing_keypoints_mask_index = np.arange(len(nk), dtype=np.int32)
        new_keypoints = new_keypoints[existing_keypoints_mask_index]
        new_des = new_des[existing_keypoints_mask_index]

        if len(new_keypoints):
            new_rays = cam.back_project_to_rays(new_keypoints)
            r0 = ekf.n_ray
            ekf.add_rays(new_rays, self.angle_var)
            self.des = np.vstack([self.des, new_des]) if len(self.des) else np.asarray(new_des, np.float64)
            keypoints_index = np.append(keypoints_index, np.arange(r0, r0 + len(new_rays)))
        keypoints = np.concatenate([keypoints.reshape(-1, 2), new_keypoints.reshape(-1, 2)], axis=0)
        return keypoints, keypoints_index

    # ------------------------------------------------------------------ ptz_slam.py:390-462
    def tracking(self, next_img, bad_tracking_percentage, bounding_box=None):
        inlier_keypoints, inlier_index, outlier_index = matching_and_ransac(
            self.previous_img, next_img, self.previous_keypoints, self.previous_keypoints_index)

        tracking_percentage = len(inlier_index) / len(self.previous_keypoints) * 100
        if tracking_percentage < bad_tracking_percentage:
            self.bad_tracking_cnt += 1
        if self.bad_tracking_cnt > 3:
            self.tracking_lost = True
            self.bad_tracking_cnt = 0

        # 1. predict: constant-velocity pose, inflate the pose covariance
        self.current_camera = copy.deepcopy(self.cameras[-1])
        self.current_camera.set_ptz(self.current_camera.get_ptz() + self.velocity)
        if not self.tracking_lost:
            self.cameras.append(self.current_camera)
        q_k = 5 * np.diag([self.angle_var, self.angle_var, self.f_var])
        self._push().add_pose_cov(q_k)

        # 2. update
        height, width = next_img.shape[0:2]
        self.ekf_update(inlier_keypoints, inlier_index, height, width)

        # 3. drop RANSAC outliers
        self.remove_rays(outlier_index)

        # 4. new features, previous frame
        self.previous_img = next_img
        self.previous_keypoints, self.previous_keypoints_index = self.add_rays(next_img, bounding_box)

        print("tracking", tracking_percentage)
        if self.keyframe_map.good_new_keyframe(self.current_camera.get_ptz(), 10, 15):
            self.new_keyframe = True

    # ------------------------------------------------------------------ ptz_slam.py:464-504
    def relocalize(self, img, camera, enable_rf=False, bounding_box=None):
        if enable_rf:
            relocalize_frame = KeyFrame(img, -1, camera.camera_center, camera.base_rotation,
                                        camera.principal_point[0], camera.principal_point[1], camera.pan, camera.tilt,
                                        camera.focal_length)
            kp, des = detect_compute_sift_array(img, 500)
            if bounding_box is not None:
                masked_index = keypoints_masking(kp, bounding_box)
                kp = kp[masked_index]
                des = des[masked_index]
            relocalize_frame.feature_pts = kp
            relocalize_frame.feature_des = des
            ptz = self.rf_map.relocalize(relocalize_frame, [camera.pan, camera.tilt, camera.focal_length])
            camera.set_ptz(ptz)
        else:
            if len(self.keyframe_map.keyframe_list) > 1:
                from relocalization import relocalization_camera
                lost_pose = camera.pan, camera.tilt, camera.focal_length
                relocalize_pose = relocalization_camera(self.keyframe_map, img, lost_pose)
                camera.set_ptz(relocalize_pose)
            else:
                print("Warning: Not enough keyframes for relocalization.")
        self.tracking_lost = False
        return camera

    # ------------------------------------------------------------------ ptz_slam.py:506-539
    def add_keyframe(self, img, camera, frame_index, enable_rf=False):
        new_keyframe = KeyFrame(img, frame_index, camera.camera_center, camera.base_rotation, camera.principal_point[0],
                                camera.principal_point[1], camera.pan, camera.tilt, camera.focal_length)
        if enable_rf:
            new_keyframe.feature_pts = self.previous_keypoints
            new_keyframe.feature_des = self.des[np.asarray(self.previous_keypoints_index).astype(int)]
            self.rf_map.add_keyframe(new_keyframe)
            self.new_keyframe = False
        else:
            if frame_index == 0:
                self.keyframe_map.add_first_keyframe(new_keyframe, verbose=True)
            else:
                self.keyframe_map.add_keyframe_with_ba(new_keyframe, "./bundle_result/", verbose=True)
                self.new_keyframe = False
