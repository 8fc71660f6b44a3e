"""A plain-Python restatement of the rectangular shortest-augmenting-path assignment that
scipy.optimize.linear_sum_assignment implements (Crouse, "On implementing 2D rectangular assignment
algorithms", IEEE TAES 2016), in float64 with scipy's tie rule -- the specification the HIP solver
(csrc/lsap.hip) follows step for step.  TEST INFRASTRUCTURE: checked against scipy itself in
tests/test_lsap.py; the product never imports it."""
import math

import numpy as np


def _augmenting_path(cost, u, v, path, row4col, spc, cur_row):
    nr, nc = cost.shape
    min_val = 0.0
    remaining = [nc - it - 1 for it in range(nc)]
    num_rem = nc
    SR = [False] * nr
    SC = [False] * nc
    for j in range(nc):
        spc[j] = math.inf
    sink = -1
    i = cur_row
    while sink == -1:
        index = -1
        lowest = math.inf
        SR[i] = True
        for it in range(num_rem):
            j = remaining[it]
            r = min_val + float(cost[i, j]) - u[i] - v[j]
            if r < spc[j]:
                path[j] = i
                spc[j] = r
            if spc[j] < lowest or (spc[j] == lowest and row4col[j] == -1):
                lowest = spc[j]
                index = it
        min_val = lowest
        if min_val == math.inf:
            raise ValueError("infeasible cost matrix")
        j = remaining[index]
        if row4col[j] == -1:
            sink = j
        else:
            i = row4col[j]
        SC[j] = True
        num_rem -= 1
        remaining[index] = remaining[num_rem]
    return sink, min_val, SR, SC


def linear_sum_assignment_ref(cost):
    """cost (n_rows, n_cols) -> (row_ind, col_ind) like scipy (rows sorted ascending)."""
    cost = np.asarray(cost, dtype=np.float64)
    transposed = cost.shape[1] < cost.shape[0]
    if transposed:
        cost = cost.T
    nr, nc = cost.shape
    u = [0.0] * nr
    v = [0.0] * nc
    spc = [0.0] * nc
    path = [-1] * nc
    col4row = [-1] * nr
    row4col = [-1] * nc
    for cur_row in range(nr):
        sink, min_val, SR, SC = _augmenting_path(cost, u, v, path, row4col, spc, cur_row)
        u[cur_row] += min_val
        for i in range(nr):
            if SR[i] and i != cur_row:
                u[i] += min_val - spc[col4row[i]]
        for j in range(nc):
            if SC[j]:
                v[j] -= min_val - spc[j]
        j = sink
        while True:
            i = path[j]
            row4col[j] = i
            col4row[i], j = j, col4row[i]
            if i == cur_row:
                break
    a = np.asarray(col4row, dtype=np.int64)
    if transposed:
        order = np.argsort(a)
        return a[order], order
    return np.arange(nr), a
