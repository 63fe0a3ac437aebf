"""Robot model fixture (decoded from zbot_6s_new.usd) vs the reference's printed known answers.

Known answers: base z 0.2545 and base quat (0.6003, -0.6003, -0.3735, -0.3739) at the default pose
(v2.py:403-404); feet z 0 / 0.053 (v4.py:816); 12 links of 0.25042 kg (zbot_6s_new.usd);
joint1.localRot0 = (0.92388, 0, 0.382683, 0)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from zbot_lab_amd import model as zm

REF_USD = "/root/reference/source/zbot/zbot/assets/zbot_assets/zbot_6s_new.usd"


def test_fk_known_answers(robot):
    _, links = robot.fk(robot.default_root_pos, robot.default_root_quat, robot.default_joint_pos)
    base = links[zm.LINK_NAMES.index("base")]
    np.testing.assert_allclose(base.p[2], 0.2545, atol=5e-5)
    np.testing.assert_allclose(base.q, [0.6003, -0.6003, -0.3735, -0.3739], atol=1e-4)
    np.testing.assert_allclose(links[0].p[2], 0.0, atol=1e-6)
    np.testing.assert_allclose(links[11].p, [0.0001, 0.06, 0.053], atol=1e-4)


def test_oracle_fk_matches_model(robot, oracle_lib):
    from oracle.pyoracle import OracleSim
    s = OracleSim(2)
    p, q = s.link_poses()
    _, links = robot.fk(robot.default_root_pos, robot.default_root_quat, robot.default_joint_pos)
    for i, l in enumerate(links):
        np.testing.assert_allclose(p[0, i], l.p, atol=2e-6)
        np.testing.assert_allclose(q[0, i], l.q, atol=2e-6)


def test_mass_properties(robot):
    assert len(robot.raw["links"]) == 12
    for l in robot.raw["links"]:
        np.testing.assert_allclose(l["mass"], 0.25042, rtol=1e-6)
    np.testing.assert_allclose(robot.body_mass.sum(), 3.00504, rtol=1e-5)
    assert robot.link_body == [0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6]
    for I in robot.body_inertia:
        assert np.linalg.eigvalsh(I).min() > 1e-5
    # authored COM used verbatim (not recomputed from geometry), SURVEY.md §8a A1
    np.testing.assert_allclose(robot.raw["links"][0]["com"], [-0.0082592, -5.1e-8, 0.028345], atol=1e-6)
    np.testing.assert_allclose(robot.raw["links"][1]["com"], [-0.011593, -5.1e-8, 0.023274], atol=1e-6)


def test_collision_shape(robot):
    for i in range(12):
        for c in range(2):
            E1, E2 = robot.circles[i, c, 3:6], robot.circles[i, c, 6:9]
            np.testing.assert_allclose(np.linalg.norm(E1), 0.05, rtol=1e-6)
            np.testing.assert_allclose(np.linalg.norm(E2), 0.05, rtol=1e-6)
            assert abs(E1 @ E2) < 1e-9
    # feet rest on the plane at the default pose: the lowest rim point is at z = 0
    _, links = robot.fk(robot.default_root_pos, robot.default_root_quat, robot.default_joint_pos)
    bodies, _ = robot.fk(robot.default_root_pos, robot.default_root_quat, robot.default_joint_pos)
    for li in (0, 11):
        b = bodies[robot.link_body[li]]
        zs = []
        for c in range(2):
            C = b.apply(robot.circles[li, c, :3])
            E1 = zm.qrot(b.q, robot.circles[li, c, 3:6])
            E2 = zm.qrot(b.q, robot.circles[li, c, 6:9])
            zs.append(C[2] - np.hypot(E1[2], E2[2]))
        assert abs(min(zs)) < 1e-4
    assert len(robot.self_pairs) == 55
    assert all(b - a >= 2 for a, b in robot.self_pairs)


def test_pack_roundtrip(robot):
    m = zm.pack_model(robot)
    assert m.num_self_pairs == 55
    assert list(m.undesired_links) == list(range(1, 11))
    assert (m.base_link, m.foot_links[0], m.foot_links[1]) == (6, 0, 11)
    c = zm.TaskCfg().pack()
    assert c.max_episode_length == 1000 and abs(c.reward_scales[5] - 0.1) < 1e-7   # step_length 5 * 0.02


@pytest.mark.skipif(not os.path.exists(REF_USD), reason="reference asset not present (GPU box)")
def test_usdc_decoder_known_answers():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    from usdc import Crate
    c = Crate(REF_USD)
    assert c.version == (0, 8, 0) and len(c.tokens) == 172
    bodies = [p for p in c.specs if "." not in p and c.get(p + ".physics:mass") is not None]
    assert len(bodies) == 12
    q = c.get("/zbot/foot_0/joint1.physics:localRot0")   # stored (x, y, z, w)
    np.testing.assert_allclose([q[3], q[0], q[1], q[2]], [0.92388, 0, 0.382683, 0], atol=1e-5)
    assert "PhysicsArticulationRootAPI" in c.get("/zbot/foot_0", "apiSchemas")["explicit"]
