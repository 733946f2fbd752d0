"""Clustering stage batch nearest centroid (stages/clustering.rs:42-63) on
the GPU vs the oracle's fixed-order restatement (bit-exact: index and f32
distance), and the stage's host loop (:65-88) end to end."""
import numpy as np
import pytest
import torch

import datagen
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("b,c,f", [(1, 1, 3), (1000, 37, 16), (5000, 300, 96), (700, 1500, 33)])
def test_nearest_centroid_bit_exact(b, c, f):
    import surfface_hip as S
    X = datagen.clustered(b + c, f, seed=b, blobs=7, dup_frac=0.02, zero_frac=0.01)
    batch, cents = X[:b], X[b:]
    gi, gd = S.nearest_centroid(torch.from_numpy(batch).cuda(), torch.from_numpy(cents).cuda())
    ri, rd = O.nearest_centroid(batch, cents)
    np.testing.assert_array_equal(gi.cpu().numpy(), ri)
    np.testing.assert_array_equal(gd.cpu().numpy().view(np.uint32), rd.view(np.uint32))


def test_ties_take_the_first_index():
    import surfface_hip as S
    cents = np.array([[1.0, 0.0], [1.0, 0.0], [0.0, 1.0]], np.float32)
    batch = np.array([[1.0, 0.0], [0.0, 1.0], [0.5, 0.5]], np.float32)
    gi, gd = S.nearest_centroid(torch.from_numpy(batch).cuda(), torch.from_numpy(cents).cuda())
    ri, rd = O.nearest_centroid(batch, cents)
    assert gi.cpu().tolist() == ri.tolist() and gi.cpu().tolist()[0] == 0
    np.testing.assert_array_equal(gd.cpu().numpy().view(np.uint32), rd.view(np.uint32))


def test_clustering_stage_host_loop():
    """ClusteringStage.execute: first item seeds, new centroid iff min
    distance >= radius and room, counts sum to N; replayed on the host with
    the oracle's distances."""
    import surfface_hip as S
    X = datagen.clustered(3000, 24, seed=3, blobs=12, dup_frac=0.0, zero_frac=0.0)
    st = S.ClusteringStage(target_centroids=40, radius=1.5, batch_size=512)
    out = st.execute(torch.from_numpy(X).cuda())
    # host replay with the oracle's nearest-centroid distances
    cents = [X[0]]
    asg = []
    for b0 in range(0, len(X), 512):
        B = X[b0:b0 + 512]
        ri, rd = O.nearest_centroid(B, np.stack(cents))
        for i in range(len(B)):
            if rd[i] < np.float32(1.5):
                asg.append(int(ri[i]))
            elif len(cents) < 40:
                cents.append(B[i])
                asg.append(len(cents) - 1)
            else:
                asg.append(int(ri[i]))
    assert out.assignments.cpu().tolist() == asg
    np.testing.assert_array_equal(out.centroids.cpu().numpy(), np.stack(cents))
    assert int(out.counts.sum()) == len(X) and len(out.counts) == len(cents)
