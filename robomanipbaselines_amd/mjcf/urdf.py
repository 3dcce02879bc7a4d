"""Serial-chain URDF reader for the arm IK model (host side).

The reference builds a Pinocchio model from envs/assets/common/robots/ur5e/ur5e.urdf
(common/body/ArmManager.py:48-71) and pre-multiplies the first joint placement by the arm root
pose read from MuJoCo (ArmManager.py:64-68, MujocoUR5eEnvBase.py:43).  Pinocchio folds fixed
joints into the placement of the next moving joint; this module restates that to produce one
(R, p) placement per revolute joint of the chain, with the joint axis expressed in its frame.
"""

import xml.etree.ElementTree as ET

import numpy as np


def rpy_matrix(r, p, y):
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def _origin(j):
    o = j.find("origin")
    xyz = np.array([float(x) for x in o.attrib.get("xyz", "0 0 0").split()]) if o is not None else np.zeros(3)
    rpy = np.array([float(x) for x in o.attrib.get("rpy", "0 0 0").split()]) if o is not None else np.zeros(3)
    T = np.eye(4)
    T[:3, :3] = rpy_matrix(*rpy)
    T[:3, 3] = xyz
    return T


def arm_chain(urdf_path, n_joints, root_pose=None):
    """Return (placements [n,4,4], axes [n,3], names) of the first n moving joints from the root
    link, with fixed joints folded in and root_pose (4x4) pre-multiplied on the first one."""
    root = ET.parse(urdf_path).getroot()
    joints = root.findall("joint")
    by_parent = {}
    for j in joints:
        by_parent.setdefault(j.find("parent").attrib["link"], []).append(j)
    children = {j.find("child").attrib["link"] for j in joints}
    links = [lk.attrib["name"] for lk in root.findall("link")]
    root_link = [lk for lk in links if lk not in children][0]
    placements, axes, names = [], [], []
    acc = np.eye(4) if root_pose is None else np.asarray(root_pose, np.float64)
    link = root_link
    while len(placements) < n_joints:
        cands = by_parent.get(link, [])
        # follow the chain: prefer a moving joint, else the fixed joint that leads to one
        nxt = None
        for j in cands:
            if j.attrib["type"] in ("revolute", "continuous", "prismatic"):
                nxt = j
                break
        if nxt is None:
            for j in cands:
                child = j.find("child").attrib["link"]
                if _leads_to_moving(child, by_parent):
                    nxt = j
                    break
        if nxt is None:
            raise ValueError("chain ended early")
        T = _origin(nxt)
        if nxt.attrib["type"] == "fixed":
            acc = acc @ T
        else:
            placements.append(acc @ T)
            a = nxt.find("axis")
            ax = np.array([float(x) for x in a.attrib.get("xyz", "1 0 0").split()]) if a is not None else np.array([1.0, 0, 0])
            axes.append(ax / np.linalg.norm(ax))
            names.append(nxt.attrib["name"])
            acc = np.eye(4)
        link = nxt.find("child").attrib["link"]
    return np.array(placements), np.array(axes), names


def _leads_to_moving(link, by_parent, depth=0):
    if depth > 64:
        return False
    for j in by_parent.get(link, []):
        if j.attrib["type"] != "fixed":
            return True
        if _leads_to_moving(j.find("child").attrib["link"], by_parent, depth + 1):
            return True
    return False
