"""
TransFunction — ray <-> image closed forms of the BA camera model, computed by libptzba on the GPU.

Same names, arguments (degrees, pixels) and return values as the reference
(slam_system/transformation.py:99-175).  Scalar calls return python floats like the reference;
array arguments are evaluated in one batched device call.  There is no CPU fallback.
"""
import numpy as np

import ptzba


def _scalar_or_array(vals):
    return all(np.ndim(v) == 0 for v in vals)


class TransFunction:
    device = 0

    @staticmethod
    def from_ray_to_image(u, v, f, c_p, c_t, p, t):
        """transformation.py:99-135: ray (theta=p, phi=t) -> image (x, y) for camera (c_p, c_t, f).
        Equivalent q form: x = u + f q0/q2, y = v + f q1/|q2|."""
        x, y = ptzba.ray_to_image(float(u), float(v), f, c_p, c_t, p, t, device=TransFunction.device)
        if _scalar_or_array((f, c_p, c_t, p, t)):
            return float(x), float(y)
        return x, y

    @staticmethod
    def from_image_to_ray(u, v, f, c_p, c_t, x, y):
        """transformation.py:137-175: image point -> ray (theta, phi) in degrees."""
        th, ph = ptzba.image_to_ray(float(u), float(v), f, c_p, c_t, x, y, device=TransFunction.device)
        if _scalar_or_array((f, c_p, c_t, x, y)):
            return float(th), float(ph)
        return th, ph

    @staticmethod
    def from_rays_to_image(u, v, f, c_p, c_t, rays):
        """Batched form: rays [n,2] -> points [n,2] (the reference's version of this helper is dead code,
        transformation.py:250-275; this one works)."""
        rays = np.asarray(rays, np.float64).reshape(-1, 2)
        x, y = ptzba.ray_to_image(float(u), float(v), np.full(len(rays), f), np.full(len(rays), c_p),
                                  np.full(len(rays), c_t), rays[:, 0], rays[:, 1], device=TransFunction.device)
        return np.stack([x, y], 1)

    @staticmethod
    def from_image_to_rays(u, v, f, c_p, c_t, points):
        pts = np.asarray(points, np.float64).reshape(-1, 2)
        n = len(pts)
        th, ph = ptzba.image_to_ray(float(u), float(v), np.full(n, f), np.full(n, c_p), np.full(n, c_t), pts[:, 0],
                                    pts[:, 1], device=TransFunction.device)
        return np.stack([th, ph], 1)
