"""CPU: host-side logic of ogbench_amd.datasets (no kernel calls)."""


def test_periodic_layout_detection():
    """datasets.periodic_layout: the closed form is accepted exactly when it
    reproduces valid_idxs and the trajectory ends (CPU tensors)."""
    import torch
    from ogbench_amd.datasets import periodic_layout

    n_traj, L = 7, 13
    R = n_traj * L
    rows = torch.arange(R)
    valid = rows[(rows % L) != L - 1]
    ends = (valid // L) * L + (L - 2)
    assert periodic_layout(R, valid, ends) == (L, L - 1, L - 2)
    # every row pickable, terminal at the last row of each trajectory
    assert periodic_layout(R, None, (rows // L) * L + (L - 1)) == (L, L, L - 1)
    # one trajectory of another length: tables
    bad = valid.clone()
    bad[20] += 1
    assert periodic_layout(R, bad, ends) == (0, 0, 0)
    bad_ends = ends.clone()
    bad_ends[-1] -= 1
    assert periodic_layout(R, valid, bad_ends) == (0, 0, 0)
    assert periodic_layout(R, None, (rows // L) * L + (L - 2)) == (0, 0, 0)
