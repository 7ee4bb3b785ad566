import sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests'); sys.path.insert(0, '/root/repo/oracle')
import bench, test_gpu_fullsize as T
knn = bench.load_knn()
DEV = torch.device('cuda', 0)
n, m, d, k = 10_000_000, 256, 96, 10
X, lab, Q, _ = bench.synth(n, m, d, 10, 2468, 1357, DEV)
w = k + 1
for (a, b) in [(0, 5_000_000), (5_000_000, 10_000_000), (0, 1_000_000), (0, 2_500_000), (0, 4_000_000)]:
    Xs, Ls = X[a:b], lab[a:b]
    c = knn.Classifier(0)
    c.set_train_device(Xs.data_ptr(), Ls.data_ptr(), b - a, d, 10, idx_offset=a, keep=(Xs, Ls))
    pd = torch.empty((m, w), dtype=torch.float64, device=DEV)
    pi = torch.empty((m, w), dtype=torch.int64, device=DEV)
    pl = torch.empty((m, w), dtype=torch.int32, device=DEV)
    c.search_partial_device(Q.data_ptr(), m, w, knn.L2, pd.data_ptr(), pi.data_ptr(), pl.data_ptr())
    c.sync()
    idx = pi.cpu().numpy(); dist = pd.cpu().numpy()
    want = T.ref_distances(X, Q, idx)
    bad = np.nonzero(want.view(np.int64) != dist.view(np.int64))
    bf = T.brute_force_kdist(Xs, Q, w)
    opt = np.abs(dist - bf).max()
    print('shard [%d,%d): rescans=%d mismatches=%d  max|d-bf|=%.3g geom=%s' % (a, b, c.last_rescan_count(), bad[0].size, opt, c.last_geometry()))
    for q, t in list(zip(*bad))[:3]:
        print('  q', q, 't', t, 'idx', idx[q, t], 'gpu %.17g host %.17g' % (dist[q, t], want[q, t]))
    c.close()
