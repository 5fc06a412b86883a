"""Host timeline of device SsTable::create calls (CB_FLUSH_TRACE=1 makes the
library print one '[flush] ...' line per call to stderr: microseconds from
entry at each step). Sorted and unsorted 1M-entry batches on a side stream,
as in bench.py's flush leg. Diagnostic only."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lsmt_amd  # noqa: E402
from lsmt_amd import workload  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.Stream(device=dev)
n = 1 << 20
fk = workload.key_range(7000, n)
fv = workload.table_value(fk, 1)
for label, keys_np in (("sorted", workload.sort_keys16(fk)), ("unsorted", fk)):
    kd = torch.from_numpy(np.ascontiguousarray(keys_np.reshape(-1))).to(dev)
    vd = torch.from_numpy(np.ascontiguousarray(fv.reshape(-1))).to(dev)
    ko = torch.from_numpy(np.arange(0, 16 * (n + 1), 16, dtype=np.int64)).to(dev)
    kb = lsmt_amd.KeyBatch(n=n, data=kd, offsets=ko)
    vb = lsmt_amd.KeyBatch(n=n, data=vd, offsets=ko)
    torch.cuda.synchronize()
    made = []
    print(label, file=sys.stderr, flush=True)
    for _ in range(12):
        made.append(lsmt_amd.sstable_create((kb, vb), m=1 << 26, device=0, stream=st.cuda_stream))
        if len(made) > 2:
            made.pop(0)
    torch.cuda.synchronize()
