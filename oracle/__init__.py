"""oracle -- TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference hot path (hliuson/ogbench), used exclusively
as the checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  The product (ogbench_amd/, libogbx.so) never imports, links or calls
anything here.  See DESIGN.md "Oracle" for what is pinned and what is not.
"""
