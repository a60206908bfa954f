"""CPU oracle for the meta-kriging hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker or the timed CPU baseline.  The shipped
library never calls it.  Parity status: see oracle/spmvglm.py header
("parity unpinned" against spBayes, which is absent; pinned against scipy and
against the literal spBayes-structured restatement in oracle/literal.py).
"""
