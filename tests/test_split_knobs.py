"""Host-side checks of the depth split's tuning knobs (include/gsr.h, GSR_TUNE_DEPTH_SPLIT*):
defaults, ranges, read-only knobs and the per-lane restart — no device work, so these run
without a GPU (the GPU behaviour is tests/test_gpu_depth_split.py)."""
import pytest

KNOB_SPLIT, KNOB_PM, KNOB_UNSAT, KNOB_STATE = 23, 24, 25, 26


def test_split_knob_defaults_and_ranges(gsr):
    r = gsr.Renderer()
    assert (gsr.TUNE_DEPTH_SPLIT, gsr.TUNE_DEPTH_SPLIT_PERMILLE, gsr.TUNE_DEPTH_SPLIT_UNSAT,
            gsr.TUNE_DEPTH_SPLIT_STATE) == (KNOB_SPLIT, KNOB_PM, KNOB_UNSAT, KNOB_STATE)
    assert r.get_tuning(KNOB_SPLIT) == 2          # on above 1.5M Gaussians
    assert r.get_tuning(KNOB_PM) == 250           # starting split point
    assert r.get_tuning(KNOB_UNSAT) == 0          # nothing rendered yet
    assert r.get_tuning(KNOB_STATE) == 0          # no split frame yet
    for v in (0, 1, 2):
        r.set_tuning(KNOB_SPLIT, v)
        assert r.get_tuning(KNOB_SPLIT) == v
    for v in (1, 138, 999):
        r.set_tuning(KNOB_PM, v)
        assert r.get_tuning(KNOB_PM) == v
    for knob, v in ((KNOB_SPLIT, -1), (KNOB_SPLIT, 3), (KNOB_PM, 0), (KNOB_PM, 1000), (KNOB_UNSAT, 0),
                    (KNOB_STATE, 0)):
        with pytest.raises(gsr.GsrError):
            r.set_tuning(knob, v)
    r.close()


def test_split_point_reaches_new_lanes(gsr):
    """Lanes created later (frames in flight) start from lane 0's split point."""
    r = gsr.Renderer()
    r.set_tuning(KNOB_PM, 123)
    r.set_frames_in_flight(4)
    assert r.frames_in_flight() == 4 and r.get_tuning(KNOB_PM) == 123
    r.close()
