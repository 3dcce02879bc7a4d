"""Data-key vocabulary (common/data/DataKey.py:4-150 of the reference) and the device routing codes
of the keys the batched UR5e rollout serves (include/rmbx.h RMBX_KEY_*).

Dimensions are those DataKey.get_dim (:94-150) gives for the UR5e envs' single ArmConfig
(envs/mujoco/ur5e/MujocoUR5eEnvBase.py:37-52: 6 arm joints, 1 gripper joint, eef_idx 0)."""


class DataKey:
    TIME = "time"
    REWARD = "reward"
    MEASURED_JOINT_POS = "measured_joint_pos"
    COMMAND_JOINT_POS = "command_joint_pos"
    MEASURED_JOINT_POS_REL = "measured_joint_pos_rel"
    COMMAND_JOINT_POS_REL = "command_joint_pos_rel"
    MEASURED_JOINT_VEL = "measured_joint_vel"
    COMMAND_JOINT_VEL = "command_joint_vel"
    MEASURED_JOINT_TORQUE = "measured_joint_torque"
    COMMAND_JOINT_TORQUE = "command_joint_torque"
    MEASURED_GRIPPER_JOINT_POS = "measured_gripper_joint_pos"
    COMMAND_GRIPPER_JOINT_POS = "command_gripper_joint_pos"
    MEASURED_EEF_POSE = "measured_eef_pose"
    COMMAND_EEF_POSE = "command_eef_pose"
    MEASURED_EEF_POSE_REL = "measured_eef_pose_rel"
    COMMAND_EEF_POSE_REL = "command_eef_pose_rel"
    MEASURED_EEF_VEL = "measured_eef_vel"
    COMMAND_EEF_VEL = "command_eef_vel"
    MEASURED_EEF_WRENCH = "measured_eef_wrench"
    COMMAND_EEF_WRENCH = "command_eef_wrench"
    MEASURED_MOBILE_OMNI_VEL = "measured_mobile_omni_vel"
    COMMAND_MOBILE_OMNI_VEL = "command_mobile_omni_vel"

    # DataKey.py:66-91
    MEASURED_DATA_KEYS = [MEASURED_JOINT_POS, MEASURED_JOINT_POS_REL, MEASURED_JOINT_VEL,
                          MEASURED_GRIPPER_JOINT_POS, MEASURED_EEF_POSE, MEASURED_EEF_POSE_REL,
                          MEASURED_EEF_WRENCH, MEASURED_MOBILE_OMNI_VEL]
    COMMAND_DATA_KEYS = [COMMAND_JOINT_POS, COMMAND_JOINT_POS_REL, COMMAND_GRIPPER_JOINT_POS,
                         COMMAND_EEF_POSE, COMMAND_EEF_POSE_REL, COMMAND_MOBILE_OMNI_VEL]

    @classmethod
    def get_dim(cls, key, env=None):
        if key == cls.TIME:
            return 1
        if key in (cls.MEASURED_JOINT_POS, cls.COMMAND_JOINT_POS, cls.MEASURED_JOINT_POS_REL,
                   cls.COMMAND_JOINT_POS_REL, cls.MEASURED_JOINT_VEL, cls.COMMAND_JOINT_VEL,
                   cls.MEASURED_JOINT_TORQUE, cls.COMMAND_JOINT_TORQUE):
            return 7
        if key in (cls.MEASURED_GRIPPER_JOINT_POS, cls.COMMAND_GRIPPER_JOINT_POS):
            return 1
        if key in (cls.MEASURED_EEF_POSE, cls.COMMAND_EEF_POSE):
            return 7
        if key in (cls.MEASURED_EEF_POSE_REL, cls.COMMAND_EEF_POSE_REL, cls.MEASURED_EEF_VEL,
                   cls.COMMAND_EEF_VEL, cls.MEASURED_EEF_WRENCH, cls.COMMAND_EEF_WRENCH):
            return 6
        if key in (cls.MEASURED_MOBILE_OMNI_VEL, cls.COMMAND_MOBILE_OMNI_VEL):
            return 3
        raise ValueError(f"[{cls.__name__}] Invalid data key: {key}")


# include/rmbx.h RMBX_KEY_*: the state keys MotionManager.get_data serves for a UR5e env
# (MotionManager.py:41-130; the *_rel measured keys fall through to its ValueError, and the UR5e
# env has no mobile base) and the command keys ArmManager.set_command_data handles (:88-123).
STATE_KEY_CODES = {
    DataKey.MEASURED_JOINT_POS: 1,
    DataKey.MEASURED_JOINT_VEL: 2,
    DataKey.MEASURED_GRIPPER_JOINT_POS: 3,
    DataKey.MEASURED_EEF_POSE: 4,
    DataKey.MEASURED_EEF_WRENCH: 5,
    DataKey.COMMAND_JOINT_POS: 16,
    DataKey.COMMAND_GRIPPER_JOINT_POS: 18,
    DataKey.COMMAND_EEF_POSE: 19,
}
ACTION_KEY_CODES = {
    DataKey.COMMAND_JOINT_POS: 16,
    DataKey.COMMAND_JOINT_POS_REL: 17,
    DataKey.COMMAND_GRIPPER_JOINT_POS: 18,
    DataKey.COMMAND_EEF_POSE: 19,
    DataKey.COMMAND_EEF_POSE_REL: 20,
}


def state_key_codes(keys):
    """Device codes of the state keys, raising ValueError where the reference's get_state would
    (MotionManager.get_data :47-52, get_measured_data :87-90, get_command_data :100-103)."""
    codes = []
    for key in keys:
        if key not in DataKey.MEASURED_DATA_KEYS and key not in DataKey.COMMAND_DATA_KEYS:
            raise ValueError(f"[MotionManager] Invalid data key: {key}")
        if key not in STATE_KEY_CODES:
            kind = "measured" if key in DataKey.MEASURED_DATA_KEYS else "command"
            raise ValueError(f"[MotionManager] Invalid {kind} data key: {key}")
        codes.append(STATE_KEY_CODES[key])
    if len(codes) > 8:
        raise ValueError(f"at most 8 state keys are routed on the device (got {len(codes)})")
    return codes


def action_key_codes(keys):
    """Device codes of the action keys, raising ValueError where MotionManager.set_command_data
    (:25-39) / ArmManager.set_command_data (:120-123) would."""
    codes = []
    for key in keys:
        if key not in ACTION_KEY_CODES:
            raise ValueError(f"[MotionManager] Command data key is not supported by any body manager: {key}")
        codes.append(ACTION_KEY_CODES[key])
    if len(codes) > 8:
        raise ValueError(f"at most 8 action keys are routed on the device (got {len(codes)})")
    return codes
