"""Host-side bookkeeping of FFMPVec.temporal_maps (no GPU): the frame history's slot list
(_note_window) against a brute-force simulation of which frame each ring slot holds, for the
seamless ring (every step writes the new frame only) and the wrapping ring (both frames at a wrap)."""
import pytest

from flow_field_based_motion_planner_amd.vec_env import FFMPVec


class _Ring:
    """The window logic of FFMPVec without a device: _next_window / _note_window / reset."""
    _next_window = FFMPVec._next_window
    _note_window = FFMPVec._note_window

    def __init__(self, W, seamless):
        self.frame_window, self.ring = W, "seamless" if seamless else "wrap"
        self._wpos, self._hist, self._hist_from_reset = 0, [], False
        self.slots = [None] * W  # frame id held by each physical slot

    def _set_window(self, p):
        self._wpos = p

    def reset(self, frame):
        self._set_window(0)
        self._hist, self._hist_from_reset = [], True
        self._note_window(True)
        self.slots[0] = self.slots[1] = frame

    def step(self, frame, prev):
        full = self._next_window()
        W = self.frame_window
        self.slots[(self._wpos + 1) % W] = frame
        if full:
            self.slots[self._wpos % W] = prev  # the older frame re-rastered from the record


@pytest.mark.parametrize("W,seamless", [(3, True), (4, True), (8, True), (3, False), (4, False), (6, False)])
def test_history_slots_hold_the_lagged_frames(W, seamless):
    r = _Ring(W, seamless)
    r.reset(0)
    for f in range(1, 40):
        r.step(f, f - 1)
        assert len(r._hist) == len(set(r._hist)) <= W
        for d, s in enumerate(r._hist):
            assert r.slots[s] == max(f - d, 0), (f, d, s, r.slots, r._hist)  # the reset frame twice
        # the guarantee that lags beyond the list are clamped away holds only until a frame is lost
        if r._hist_from_reset:
            assert len(r._hist) == f + 2
    # a seamless ring keeps all W frames, a wrapping one W - 1 after its first wrap
    assert len(r._hist) >= (W if seamless else W - 1)
