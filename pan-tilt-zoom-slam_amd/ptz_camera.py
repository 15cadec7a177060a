"""
PTZCamera (reference: slam_system/ptz_camera.py:16-325) — same constructor, attributes and methods.

Projection / back-projection of rays (the EKF tracking model: signed q2, optional 6-parameter
displacement between rotation and projection centre, ptz_camera.py:106-115, 191-325) run on the GPU
through libptzba (batched); the 3x3 matrix accessors are plain host bookkeeping.
The 3-D-point methods (project_3d_point, back_project_to_3d_point) serve the offline calibration
path, which is out of scope.
"""
import math

import numpy as np

import ptzba


class PTZCamera:
    device = 0

    def __init__(self, principal_point, camera_center, base_rotation, displacement=None):
        if displacement is not None:
            assert len(displacement) == 6
        self.principal_point = principal_point
        self.camera_center = camera_center
        base_rotation = np.asarray(base_rotation, np.float64)
        assert base_rotation.shape == (3, 3) or base_rotation.shape == (3,)
        if base_rotation.shape == (3, 3):
            self.base_rotation = base_rotation
        else:
            self.base_rotation = _rodrigues(base_rotation)
        self.pan = 0.0
        self.tilt = 0.0
        self.focal_length = 2000
        self.displacement = np.zeros(6) if displacement is None else np.asarray(displacement, np.float64)
        self.projection_matrix = np.zeros((3, 4))

    # ---------------- matrices (ptz_camera.py:55-141) ----------------
    def compute_camera_matrix(self):
        return np.array([[self.focal_length, 0, self.principal_point[0]], [0, self.focal_length, self.principal_point[1]],
                         [0, 0, 1]])

    def compute_pan_matrix(self):
        p = math.radians(self.pan)
        return np.array([[math.cos(p), 0, -math.sin(p)], [0, 1, 0], [math.sin(p), 0, math.cos(p)]])

    def compute_tilt_matrix(self):
        t = math.radians(self.tilt)
        return np.array([[1, 0, 0], [0, math.cos(t), math.sin(t)], [0, -math.sin(t), math.cos(t)]])

    def compute_rotation_matrix(self):
        return self.compute_tilt_matrix() @ self.compute_pan_matrix() @ self.base_rotation

    def compute_dispalcement(self):  # (sic) reference name, ptz_camera.py:106
        fl, w = self.focal_length, self.displacement
        return np.array([w[0] + w[3] * fl, w[1] + w[4] * fl, w[2] + w[5] * fl])

    compute_displacement = compute_dispalcement

    def recompute_matrix(self):
        K = self.compute_camera_matrix()
        cc = np.identity(4)
        cc[0:3, 3] = -np.asarray(self.camera_center, np.float64)
        R = np.identity(4)
        R[0:3, 0:3] = self.compute_rotation_matrix()
        d = np.eye(3, 4)
        d[:, 3] = self.compute_dispalcement()
        self.projection_matrix = K @ d @ R @ cc

    def get_ptz(self):
        return np.array([self.pan, self.tilt, self.focal_length])

    def set_ptz(self, ptz):
        self.pan, self.tilt, self.focal_length = ptz
        self.recompute_matrix()

    def _disp(self):
        return self.displacement if np.any(self.displacement != 0) else None

    # ---------------- rays (GPU) ----------------
    def project_ray(self, ray):
        """ptz_camera.py:191-210: one ray -> (x, y)."""
        xy = ptzba.project_rays(self.principal_point[0], self.principal_point[1], self.focal_length, self.pan, self.tilt,
                                np.asarray(ray, np.float64).reshape(1, 2), self._disp(), device=PTZCamera.device)
        return float(xy[0, 0]), float(xy[0, 1])

    def project_rays(self, rays, height=0, width=0):
        """ptz_camera.py:212-234: [n,2] rays -> (points [m,2], float index [m]); with height/width only
        rays strictly inside the image (0<x<w, 0<y<h) are returned."""
        rays = np.asarray(rays, np.float64).reshape(-1, 2)
        if len(rays) == 0:
            return np.ndarray([0, 2], np.float32), np.ndarray([0])
        pts = ptzba.project_rays(self.principal_point[0], self.principal_point[1], self.focal_length, self.pan,
                                 self.tilt, rays, self._disp(), device=PTZCamera.device)
        if height != 0 and width != 0:
            keep = (pts[:, 0] > 0) & (pts[:, 0] < width) & (pts[:, 1] > 0) & (pts[:, 1] < height)
            return pts[keep], np.flatnonzero(keep).astype(np.float64)
        return pts, np.ndarray([0])

    def back_project_to_ray(self, x, y):
        """ptz_camera.py:287-312."""
        r = ptzba.back_project_rays(self.principal_point[0], self.principal_point[1], self.focal_length, self.pan,
                                    self.tilt, np.array([[x, y]], np.float64), self._disp(), device=PTZCamera.device)
        return float(r[0, 0]), float(r[0, 1])

    def back_project_to_rays(self, points):
        """ptz_camera.py:314-325: [n,2] points -> [n,2] rays."""
        pts = np.asarray(points, np.float64).reshape(-1, 2)
        if len(pts) == 0:
            return np.ndarray([0, 2])
        return ptzba.back_project_rays(self.principal_point[0], self.principal_point[1], self.focal_length, self.pan,
                                       self.tilt, pts, self._disp(), device=PTZCamera.device)


def _rodrigues(rvec):
    rvec = np.asarray(rvec, np.float64).reshape(3)
    th = np.linalg.norm(rvec)
    if th < 1e-15:
        return np.eye(3)
    k = rvec / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * (K @ K)
