"""The restated grader awards 90/90 to the golden dbg.logs (as the reference grader does)."""
import pytest

from golden_util import load_case
from grader import grade


@pytest.mark.parametrize("seed", ["T1_R1", "T4_R2", "T8_R3", "T42_R7"])
def test_golden_scores_full_marks(seed):
    total = sum(grade(load_case(f"{c}_{seed}")["dbg"], c)
                for c in ("singlefailure", "multifailure", "msgdropsinglefailure"))
    assert total == 90
