"""Decode the reference robot asset into the committed model fixture (build container only).

Reads ``/root/reference/source/zbot/zbot/assets/zbot_assets/zbot_6s_new.usd`` (the asset that
``ZBOT_6S_CFG`` spawns, ``source/zbot/zbot/assets/zbot_cfg.py:621-669``) with the offline crate
reader in ``tools/usdc.py`` and writes ``zbot_lab_amd/assets/zbot6s_model.json``:

* per link: authored mass, COM, principal inertia + principal axes (used verbatim, as PhysX does),
  rest transform, collider orientation;
* per link collision shape: the authored ``convexHull`` collider is, to within 2 mm, the convex
  hull of two radius-5 cm circles (the module's flat base disk and its 45-degree joint disk). We
  store the two circles (centre, normal, radius) in the link frame. The fit is checked here
  against the cooked-hull input points (max deviation printed and asserted);
* per link: two self-collision spheres (a symmetric pair fitted to the same shape);
* joints: body0/body1, localPos0/1, localRot0/1 (converted to wxyz), axis;
* the spawn/actuator/init-state constants of ``ZBOT_6S_CFG`` (transcribed with file:line).

Run: ``python tools/extract_model.py`` (needs /root/reference; the GPU box never runs this).
"""
from __future__ import annotations

import json
import os
import sys
from collections import Counter

import numpy as np
from scipy.spatial import ConvexHull

sys.path.insert(0, os.path.dirname(__file__))
from usdc import Crate  # noqa: E402

REF_USD = "/root/reference/source/zbot/zbot/assets/zbot_assets/zbot_6s_new.usd"
OUT = os.path.join(os.path.dirname(__file__), "..", "zbot_lab_amd", "assets", "zbot6s_model.json")

# Isaac Lab body order = PhysX articulation link order from the root.
LINKS = ["foot_0", "b1", "a2", "b2", "a3", "b3", "base", "b4", "a5", "b5", "a6", "foot_1"]
MODULE_RADIUS = 0.05


def wxyz(q_xyzw):
    x, y, z, w = [float(v) for v in q_xyzw]
    return [w, x, y, z]


def quat_to_mat(q):
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def fit_circle(P, n):
    """Least-squares circle in the plane with normal n; iteratively trims off-circle points."""
    n = n / np.linalg.norm(n)
    e1 = np.cross(n, [0.0, 1.0, 0.0])
    if np.linalg.norm(e1) < 1e-6:
        e1 = np.cross(n, [1.0, 0.0, 0.0])
    e1 /= np.linalg.norm(e1)
    e2 = np.cross(n, e1)
    U, V = P @ e1, P @ e2
    # RANSAC over point triples (deterministic seed): the face polygon also holds points of the
    # ruled side surface, so take the circumcircle with most inliers, then refine by least squares.
    rng = np.random.default_rng(0)
    best = None
    for _ in range(3000):
        i, j, k = rng.choice(len(P), 3, replace=False)
        A = np.array([[2 * (U[j] - U[i]), 2 * (V[j] - V[i])], [2 * (U[k] - U[i]), 2 * (V[k] - V[i])]])
        if abs(np.linalg.det(A)) < 1e-12:
            continue
        b = np.array([U[j] ** 2 - U[i] ** 2 + V[j] ** 2 - V[i] ** 2, U[k] ** 2 - U[i] ** 2 + V[k] ** 2 - V[i] ** 2])
        cu, cv = np.linalg.solve(A, b)
        r = np.hypot(U[i] - cu, V[i] - cv)
        inl = np.abs(np.hypot(U - cu, V - cv) - r) < 3e-4
        if best is None or inl.sum() > best.sum():
            best = inl
    keep = best
    u, v = U[keep], V[keep]
    A = np.c_[2 * u, 2 * v, np.ones_like(u)]
    sol = np.linalg.lstsq(A, u * u + v * v, rcond=None)[0]
    cu, cv = sol[:2]
    r = np.sqrt(sol[2] + cu * cu + cv * cv)
    res = np.abs(np.hypot(U - cu, V - cv) - r)
    C = cu * e1 + cv * e2 + float(np.mean(P @ n)) * n
    return C, float(r), float(res[keep].max())


def mesh_circles(points):
    """The two largest planar faces of the hull -> two circles (centre, outward normal, radius)."""
    h = ConvexHull(points)
    hv = points[h.vertices]
    cnt = Counter(map(tuple, np.round(h.equations, 4)))
    circles = []
    for plane, _ in cnt.most_common(2):
        plane = np.array(plane)
        on = np.abs(hv @ plane[:3] + plane[3]) < 2e-4
        C, r, res = fit_circle(hv[on], plane[:3])
        circles.append({"center": C, "normal": plane[:3] / np.linalg.norm(plane[:3]), "radius": r,
                        "fit_residual": res})
    return circles, h


def circle_hull_points(circles, n=512):
    out = []
    for c in circles:
        nrm = c["normal"]
        e1 = np.cross(nrm, [0.0, 1.0, 0.0])
        if np.linalg.norm(e1) < 1e-6:
            e1 = np.cross(nrm, [1.0, 0.0, 0.0])
        e1 /= np.linalg.norm(e1)
        e2 = np.cross(nrm, e1)
        th = np.linspace(0, 2 * np.pi, n, endpoint=False)
        out.append(c["center"] + c["radius"] * (np.outer(np.cos(th), e1) + np.outer(np.sin(th), e2)))
    return np.vstack(out)


def fit_sphere_pair(circles, rng_seed=0):
    """Symmetric sphere pair (mirror plane through both circle centres) maximising IoU."""
    S = circle_hull_points(circles, 256)
    hs = ConvexHull(S)
    rng = np.random.default_rng(rng_seed)
    lo, hi = S.min(0) - 0.005, S.max(0) + 0.005
    X = rng.uniform(lo, hi, size=(20000, 3))
    inside = np.max(hs.equations[:, :3] @ X.T + hs.equations[:, 3:4], axis=0) <= 0
    c0, c1 = circles[0]["center"], circles[1]["center"]
    n0, n1 = circles[0]["normal"], circles[1]["normal"]
    mid = 0.5 * (c0 + c1)
    # in-shape frame: ey = normal of the mirror plane (spanned by the two normals)
    ey = np.cross(n0, n1)
    ey /= np.linalg.norm(ey)
    ez = (c1 - c0) / np.linalg.norm(c1 - c0)
    ex = np.cross(ey, ez)
    best = None
    # inscribed spheres only: a sphere protruding from the hull would report self contacts that
    # PhysX (exact hulls) does not, e.g. between the hip links at the default pose
    for ax in np.linspace(-0.02, 0.02, 17):
        for az in np.linspace(-0.02, 0.02, 17):
            for ay in np.linspace(0.0, 0.025, 11):
                cs = [mid + ax * ex + az * ez + s * ay * ey for s in (1, -1)]
                r = float(min(-np.max(hs.equations[:, :3] @ c + hs.equations[:, 3]) for c in cs))
                if r <= 0.005:
                    continue
                m = np.zeros(len(X), bool)
                for c in cs:
                    m |= np.linalg.norm(X - c, axis=1) < r
                iou = (m & inside).sum() / max((m | inside).sum(), 1)
                if best is None or iou > best[0]:
                    best = (iou, cs, r)
    return best


# ZBOT_6S_V2_CFG (zbot_cfg.py:959-1005) on zbot_6s_v09.usd, the manager-based env's robot: the same
# 12 modules re-rooted at the base (two 3-joint branches); links listed here in chain order
# foot0 -> foot1 so that the simulator's serial-chain model can be built from it (model.py).
V09_USD = "/root/reference/source/zbot/zbot/assets/zbot_assets/zbot_6s_v09.usd"
V09_OUT = os.path.join(os.path.dirname(__file__), "..", "zbot_lab_amd", "assets", "zbot6s_v09_model.json")
V09_LINKS = ["foot0", "a3", "b2", "a2", "b1", "base", "a7", "b7", "a8", "b8", "a9", "foot1"]
V09_CFG = {
    # zbot_cfg.py:978-993 init_state (the articulation root is the base link)
    "root_link": "base",
    "root_pos": [0.0, 0.0, 0.2545],
    "root_rot_wxyz": [1.0, 0.0, 0.0, 0.0],
    "joint_pos": {"joint1": 2.02, "joint2": -0.837, "joint3": -0.312, "joint7": -2.02, "joint8": 0.837,
                  "joint9": 0.312},
    # zbot_cfg.py:995-1004 ImplicitActuatorCfg
    "stiffness": 20.0, "damping": 0.5, "effort_limit": 20.0, "velocity_limit": 10.0,
    # zbot_cfg.py:960-976 spawn props
    "max_depenetration_velocity": 1.0, "linear_damping": 0.0, "angular_damping": 0.0,
    "enabled_self_collisions": True, "solver_position_iteration_count": 4,
    "solver_velocity_iteration_count": 0,
}


def main(usd: str = REF_USD, link_names: list = LINKS, out: str = OUT, cfg: dict | None = None,
         source_cfg: str = "source/zbot/zbot/assets/zbot_cfg.py:621-669 (ZBOT_6S_CFG)"):
    c = Crate(usd)
    links = []
    shape_cache = {}
    for name in link_names:
        p = f"/zbot/{name}"
        col = f"{p}/collisions"
        pts = np.array(c.get(col + ".points"), dtype=np.float64)
        col_q = wxyz(c.get(col + ".xformOp:orient"))
        assert c.get(col + ".physics:approximation") == "convexHull"
        key = pts.tobytes()
        if key not in shape_cache:
            circles, hull = mesh_circles(pts)
            for ci in circles:
                assert abs(ci["radius"] - MODULE_RADIUS) < 2e-4, ci
            S = circle_hull_points(circles)
            sh = ConvexHull(S)
            dev_out = np.max(sh.equations[:, :3] @ pts[hull.vertices].T + sh.equations[:, 3:4], axis=0).max()
            assert dev_out < 2.5e-3, dev_out
            iou, sph, sr = fit_sphere_pair(circles)
            shape_cache[key] = (circles, hull.volume, sh.volume, dev_out, sph, sr, iou)
            print(f"{name}: hull nv={len(hull.vertices)} vol={hull.volume:.4e} two-circle vol={sh.volume:.4e} "
                  f"mesh outside by {dev_out * 1e3:.2f} mm; sphere pair r={sr:.4f} IoU={iou:.3f}")
        circles, vol, cvol, dev, sph, sr, iou = shape_cache[key]
        Rc = quat_to_mat(col_q)
        link = {
            "name": name,
            "mass": float(c.get(p + ".physics:mass")),
            "com": [float(v) for v in c.get(p + ".physics:centerOfMass")],
            "diag_inertia": [float(v) for v in c.get(p + ".physics:diagonalInertia")],
            "principal_axes_wxyz": wxyz(c.get(p + ".physics:principalAxes")),
            "rest_translate": [float(v) for v in c.get(p + ".xformOp:translate")],
            "rest_orient_wxyz": wxyz(c.get(p + ".xformOp:orient")),
            "collider_orient_wxyz": col_q,
            "hull_volume": vol,
            "circles": [{"center": (Rc @ ci["center"]).tolist(), "normal": (Rc @ ci["normal"]).tolist(),
                         "radius": MODULE_RADIUS} for ci in circles],
            "spheres": [{"center": (Rc @ s).tolist(), "radius": float(sr)} for s in sph],
            "articulation_root": "PhysicsArticulationRootAPI" in (c.get(p, "apiSchemas") or {}).get("explicit", []),
        }
        links.append(link)

    joints = []
    for path, spec in c.specs.items():
        if "." in path:
            continue
        t = c.get(path, "typeName")
        if t not in ("PhysicsRevoluteJoint", "PhysicsFixedJoint"):
            continue
        j = {
            "name": path.split("/")[-1],
            "type": "revolute" if t == "PhysicsRevoluteJoint" else "fixed",
            "body0": c.get(path + ".physics:body0", "targetPaths")["explicit"][0].split("/")[-1],
            "body1": c.get(path + ".physics:body1", "targetPaths")["explicit"][0].split("/")[-1],
            "local_pos0": [float(v) for v in c.get(path + ".physics:localPos0")],
            "local_rot0_wxyz": wxyz(c.get(path + ".physics:localRot0")),
            "local_pos1": [float(v) for v in c.get(path + ".physics:localPos1")],
            "local_rot1_wxyz": wxyz(c.get(path + ".physics:localRot1")),
        }
        if j["type"] == "revolute":
            j["axis"] = c.get(path + ".physics:axis")
        joints.append(j)
    joints.sort(key=lambda j: min(link_names.index(j["body0"]), link_names.index(j["body1"])))

    model = {
        "source": {
            "usd": os.path.relpath(usd, "/root/reference") + " (USDC crate 0.8.0)",
            "cfg": source_cfg,
            "tool": "tools/extract_model.py",
        },
        "links": links,
        "joints": joints,
        "cfg": cfg if cfg is not None else {
            # zbot_cfg.py:641-656 init_state
            "root_pos": [0.0, -0.06, 0.0],
            "root_rot_wxyz": [1.0, 0.0, 0.0, 0.0],
            "joint_pos": {"joint1": 0.312, "joint2": 0.837, "joint3": -2.02, "joint4": 2.02,
                          "joint5": -0.837, "joint6": -0.312},
            # zbot_cfg.py:658-668 ImplicitActuatorCfg
            "stiffness": 50.0, "damping": 5.0, "effort_limit": 20.0, "velocity_limit": 20.0,
            # zbot_cfg.py:626-639 spawn props
            "max_depenetration_velocity": 1.0, "linear_damping": 0.0, "angular_damping": 0.0,
            "enabled_self_collisions": True, "solver_position_iteration_count": 4,
            "solver_velocity_iteration_count": 0,
        },
    }
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(model, f, indent=1)
    print("wrote", os.path.normpath(out))


if __name__ == "__main__":
    if "--v09" in sys.argv:
        main(V09_USD, V09_LINKS, V09_OUT, V09_CFG, "source/zbot/zbot/assets/zbot_cfg.py:959-1005 (ZBOT_6S_V2_CFG)")
    else:
        main()
