"""Heavy hitters end to end on an MI355X: both servers'
key batches evaluated level by level with EvaluateUntilBatchSumToDevice over
the full 61-level 128-bit hierarchy; at every level the two servers' sums must
reconstruct the plaintext prefix histogram of the clients exactly, and the
final candidates must contain the heaviest values."""
import numpy as np
import pytest

from distributed_point_functions_amd import dpf as D
from distributed_point_functions_amd import heavy_hitters as HH

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_keys,top_k", [(3000, 64), (257, 1024)])
def test_heavy_hitters_reconstructs_plaintext(n_keys, top_k):
    import torch
    logs = HH.hierarchy()
    dpf = HH.create_dpf(logs)
    values, idx, alphas = HH.client_values(n_keys, seed=n_keys, distinct=512)
    seeds = np.random.default_rng(7).integers(0, 2**64, size=(2 * n_keys, 2), dtype=np.uint64)
    beta = D.to_value(HH.value_type(), HH.BETA)
    b0, b1 = dpf.generate_key_batch(alphas, [beta] * len(logs), root_seeds=seeds, threads=8)
    servers = [HH.Server(dpf, dpf.upload_key_batch(b), 4 * top_k + 256, torch.device("cuda"))
               for b in (b0, b1)]
    rec = []
    final = HH.run(dpf, servers, logs, top_k=top_k, record=rec)
    assert len(rec) == len(logs) == 61
    HH.verify(rec, logs, values, idx)
    ref = HH.plaintext_prefix_counts(values, idx, 128)
    # Pruning to the top-k prefixes per level can drop values whose ancestors
    # were outweighed, but never the Zipf head.
    head = sorted(ref, key=lambda v: (-ref[v], v))[:3]
    assert set(head) <= set(final) and len(final) == min(top_k, len(ref))
    # a second pass on reset contexts gives the same answer
    for s in servers:
        s.reset()
    assert HH.run(dpf, servers, logs, top_k=top_k) == final
