"""Where an env-step's time goes: HIP events recorded at phase boundaries on the current stream.

`mark(label)` records an event and starts `label`'s segment; each segment runs until the next mark,
so the segments tile the marked window and their sum is the window's GPU time.  The rollout base
marks policy / render / physics / glue (common/rollout_base.py, envs/ur5e_base.py) when a timer is
attached; recording an event costs a few microseconds of host time and never waits on the device.
"""

import torch


class PhaseTimer:
    def __init__(self):
        self.marks = []  # (label, event)

    def mark(self, label):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.marks.append((label, e))

    def summary(self):
        """({label: ms summed over its segments}, ms from the first mark to the last)."""
        if len(self.marks) < 2:
            return {}, 0.0
        self.marks[-1][1].synchronize()
        out = {}
        for (label, e0), (_, e1) in zip(self.marks, self.marks[1:]):
            out[label] = out.get(label, 0.0) + e0.elapsed_time(e1)
        return out, self.marks[0][1].elapsed_time(self.marks[-1][1])
