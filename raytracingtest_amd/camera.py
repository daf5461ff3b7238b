"""Unity-equivalent camera and light uniforms for the ray kernel.

The reference feeds `_camera.cameraToWorldMatrix` and
`_camera.projectionMatrix.inverse` (RaytracingMaster.cs:33-34) into
CreateCameraRay (RaytraceCompute.compute:129-141).  Unity is absent here, so
the matrices are restated: GL perspective (Matrix4x4.Perspective), camera to
world = TRS(position, rotation, 1) * Scale(1, 1, -1).  They are computed in
float64 and rounded to float32 once; the kernel and the oracle consume the
same float32 matrices, so this boundary does not affect kernel/oracle parity
(it is "parity unpinned" against Unity itself).

Scene constants (Assets/Scenes/Main.unity): vertical FOV 105.2, near 0.3,
far 1000 (:366-368); camera at (1,1,1) with identity rotation (:392-394);
directional light rotation (0.5875782, -0.23709337, 0.11933274, 0.7643941),
intensity 1 (:469,525).
"""
from dataclasses import dataclass, field

import numpy as np

MAIN_FOV = 105.2
MAIN_NEAR = 0.3
MAIN_FAR = 1000.0
MAIN_POSITION = (1.0, 1.0, 1.0)
MAIN_LIGHT_ROTATION = (0.5875782, -0.23709337, 0.11933274, 0.7643941)   # x, y, z, w
MAIN_LIGHT_INTENSITY = 1.0
OVERVIEW_EYE = (0.0, 20.0, -40.0)
OVERVIEW_TARGET = (0.0, 0.0, 0.0)
# Benchmark camera: inside the top of the [-16, 16]^3 world cube, above the
# Custom1 terrain (surface at world y ~ -9..13), looking 53 degrees down.  With
# the scene's 105.2-degree vertical FOV about 40% of the primary rays hit the
# terrain; the rest leave the cube (sky).
FLYOVER_EYE = (0.0, 15.0, -10.0)
FLYOVER_TARGET = (0.0, -6.0, 6.0)
# Terrain-facing camera (the large configs were benched only on
# the sky-heavy overview pose): above the middle of the cube looking steeply down,
# so nearly every primary ray ends on the terrain.
TERRAIN_EYE = (0.0, 14.0, -3.0)
TERRAIN_TARGET = (0.0, -10.0, 3.0)


def perspective(fov_deg, aspect, near, far):
    """Unity Matrix4x4.Perspective (OpenGL convention)."""
    cot = 1.0 / np.tan(np.deg2rad(fov_deg) * 0.5)
    m = np.zeros((4, 4))
    m[0, 0] = cot / aspect
    m[1, 1] = cot
    m[2, 2] = (far + near) / (near - far)
    m[2, 3] = 2.0 * far * near / (near - far)
    m[3, 2] = -1.0
    return m


def quat_to_matrix(q):
    x, y, z, w = q
    n = np.sqrt(x * x + y * y + z * z + w * w)
    x, y, z, w = x / n, y / n, z / n, w / n
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def look_rotation(forward, up=(0.0, 1.0, 0.0)):
    """Rotation matrix of Unity Quaternion.LookRotation(forward, up) (columns right, up, forward)."""
    f = np.asarray(forward, float)
    f = f / np.linalg.norm(f)
    r = np.cross(np.asarray(up, float), f)
    r = r / np.linalg.norm(r)
    u = np.cross(f, r)
    return np.column_stack([r, u, f])


@dataclass
class Camera:
    position: tuple = MAIN_POSITION
    rotation: np.ndarray = field(default_factory=lambda: np.eye(3))
    fov: float = MAIN_FOV
    near: float = MAIN_NEAR
    far: float = MAIN_FAR

    def camera_to_world(self):
        m = np.eye(4)
        m[:3, :3] = self.rotation
        m[:3, 3] = self.position
        return m @ np.diag([1.0, 1.0, -1.0, 1.0])

    def projection(self, width, height):
        return perspective(self.fov, width / height, self.near, self.far)

    def uniforms(self, width, height):
        """(c2w, inv_proj) as float32 4x4 in mathematical (row, column) order."""
        c2w = self.camera_to_world().astype(np.float32)
        inv_proj = np.linalg.inv(self.projection(width, height)).astype(np.float32)
        return c2w, inv_proj


def main_camera():
    """Main.unity camera pose."""
    return Camera()


def overview_camera(eye=OVERVIEW_EYE, target=OVERVIEW_TARGET):
    """'Overview' benchmark camera."""
    f = np.asarray(target, float) - np.asarray(eye, float)
    return Camera(position=tuple(eye), rotation=look_rotation(f))


def flyover_camera():
    """Bench camera for the terrain configs (C3-C5): the survey's 'overview' pose
    frames the whole cube in ~11% of the frame (3% of primary rays hit), a
    sky-dominated load; this pose puts the terrain under ~40% of the pixels."""
    return overview_camera(FLYOVER_EYE, FLYOVER_TARGET)


def terrain_camera():
    """Terrain-facing pose: nearly all primary rays hit (C4 / C5 beside 'overview')."""
    return overview_camera(TERRAIN_EYE, TERRAIN_TARGET)


CAMERAS = {"main": main_camera, "overview": overview_camera, "flyover": flyover_camera, "terrain": terrain_camera}


def main_light():
    """_DirectionalLight = (transform.forward, intensity) (RaytracingMaster.cs:36-37)."""
    fwd = quat_to_matrix(MAIN_LIGHT_ROTATION) @ np.array([0.0, 0.0, 1.0])
    return np.array([fwd[0], fwd[1], fwd[2], MAIN_LIGHT_INTENSITY], np.float32)


def column_major(m):
    """Unity Matrix4x4 memory order (what SetMatrix / the C-ABI take)."""
    return np.ascontiguousarray(np.asarray(m, np.float32).T.reshape(-1))


def pan_cameras(name, n, step_rad=0.002, radius=3.0):
    """A slow pan from camera pose `name`: frame k's eye circles the pose's eye in the xz plane by
    k * step_rad (radius `radius` world units) and looks at the pose's target (overview / flyover /
    terrain: their look-at target; main: 10 units along its forward axis).  Frame 0 is the pose
    itself.  The interactive drop-in case: a new view every frame (RaytracingMaster.cs:44-47, 55-74)."""
    base = CAMERAS[name]()
    targets = {"overview": OVERVIEW_TARGET, "flyover": FLYOVER_TARGET, "terrain": TERRAIN_TARGET}
    eye = np.asarray(base.position, float)
    target = np.asarray(targets[name], float) if name in targets else eye + 10.0 * np.asarray(base.rotation)[:, 2]
    out = []
    for k in range(n):
        a = step_rad * k
        e = eye + radius * np.array([np.sin(a), 0.0, 1.0 - np.cos(a)])
        out.append(Camera(position=tuple(e), rotation=look_rotation(target - e), fov=base.fov, near=base.near,
                          far=base.far))
    return out


def jitter_offsets(n, seed=0x5EED):
    """Seeded _PixelOffset sequence for jittered runs (RaytracingMaster.cs:35 uses Random.value)."""
    rng = np.random.default_rng(seed)
    return rng.random((n, 2)).astype(np.float32)
