"""Data-key vocabulary (common/data/DataKey.py:4-150 of the reference), the subset the rollout
path routes: measured/command joint positions (arm 6 + gripper 1)."""


class DataKey:
    TIME = "time"
    REWARD = "reward"
    MEASURED_JOINT_POS = "measured_joint_pos"
    COMMAND_JOINT_POS = "command_joint_pos"
    MEASURED_JOINT_VEL = "measured_joint_vel"
    MEASURED_GRIPPER_JOINT_POS = "measured_gripper_joint_pos"
    COMMAND_GRIPPER_JOINT_POS = "command_gripper_joint_pos"
    MEASURED_EEF_WRENCH = "measured_eef_wrench"

    @classmethod
    def get_dim(cls, key, env=None):
        if key in (cls.MEASURED_JOINT_POS, cls.COMMAND_JOINT_POS, cls.MEASURED_JOINT_VEL):
            return 7
        if key in (cls.MEASURED_GRIPPER_JOINT_POS, cls.COMMAND_GRIPPER_JOINT_POS):
            return 1
        if key == cls.MEASURED_EEF_WRENCH:
            return 6
        if key == cls.TIME:
            return 1
        raise ValueError(f"[{cls.__name__}] Invalid data key: {key}")
