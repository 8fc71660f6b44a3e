"""The GPU set matcher (csrc/lsap.hip) returns scipy.optimize.linear_sum_assignment's matching bit for bit:
random costs, tie-heavy integer costs, duplicated targets (exactly equal cost columns), videos without
events, and the largest PDVC problem (Q = 300 queries x 30 events)."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment

pytestmark = pytest.mark.gpu


def solve_both(costs, sizes):
    from pdvc.matcher import HungarianMatcher
    P, Q, E = costs.shape
    m = HungarianMatcher.solve_device(torch.from_numpy(costs).cuda(), sizes,
                                      torch.tensor(sizes, dtype=torch.int32, device="cuda"))
    got = m.host()
    for p in range(P):
        i, j = linear_sum_assignment(costs[p, :, :sizes[p]])
        assert got[p][0].tolist() == i.tolist(), (p, got[p][0].tolist(), i.tolist())
        assert got[p][1].tolist() == j.tolist(), (p, got[p][1].tolist(), j.tolist())


@pytest.mark.parametrize("kind", ["random", "ties", "duplicates"])
def test_lsap_matches_scipy(kind):
    rng = np.random.RandomState({"random": 0, "ties": 1, "duplicates": 2}[kind])
    P, Q, E = 64, 100, 12
    if kind == "ties":
        costs = rng.randint(0, 4, size=(P, Q, E)).astype(np.float32)
    else:
        costs = rng.randn(P, Q, E).astype(np.float32)
    if kind == "duplicates":
        costs[:, :, 3] = costs[:, :, 0]
        costs[:, :, 7] = costs[:, :, 0]
    sizes = [int(x) for x in rng.randint(0, E + 1, size=P)]
    sizes[0], sizes[1] = 0, E
    solve_both(costs, sizes)


def test_lsap_largest_problem():
    rng = np.random.RandomState(5)
    costs = rng.randn(4, 300, 30).astype(np.float32)
    solve_both(costs, [30, 29, 1, 17])


def test_lsap_pdvc_cost_matrices():
    """Costs from the actual matcher on a synthetic batch (with its real value distribution)."""
    from pdvc.matcher import HungarianMatcher, padded_targets
    torch.manual_seed(0)
    N, Q = 16, 100
    targets = []
    for v in range(N):
        e = 1 + v % 10
        c = torch.rand(e) * 0.8 + 0.1
        targets.append({"labels": torch.zeros(e, dtype=torch.long), "boxes": torch.stack([c, torch.rand(e) * 0.2 + 0.05], -1)})
    pt = padded_targets(targets, "cuda")
    m = HungarianMatcher(cost_class=2, cost_bbox=0, cost_giou=4)
    costs = m.cost_padded(torch.randn(N, Q, 1, device="cuda"), torch.rand(N, Q, 2, device="cuda"), pt)
    solve_both(costs.cpu().numpy(), pt["sizes"])
