"""Run the MLP-probed pipeline (lira_amd.search.ProbePipeline) of one config a
few times, for rocprofv3 --kernel-trace --stats.
usage: python tools/pipeline_prof.py <config> <data> [max_probe] [reps] [expect_probes]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lira-ann-search_amd"))
import torch  # noqa: E402

from lira_amd import PartitionedIndex, centroid_dist  # noqa: E402
from lira_amd.probing import MLP_2_Input, fit_probe_to_nearest, standard_scaler  # noqa: E402
from lira_amd.search import ProbePipeline  # noqa: E402
from lira_amd.synthetic import CONFIGS, workload  # noqa: E402

cfg, data = sys.argv[1], sys.argv[2]
N, d, B, nprobe, k, metric, nq = CONFIGS[cfg]
maxp = int(sys.argv[3]) if len(sys.argv) > 3 else B
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
hint = int(sys.argv[5]) if len(sys.argv) > 5 else 0
dev = torch.device("cuda", 0)
x, c, assign, mq = workload(cfg, 1234, dev, data)
idx = PartitionedIndex(d, metric, 0).build(assign[:, None] if assign.dim() == 1 else assign, x, B)
mean, scale = standard_scaler(centroid_dist(x[:65536].contiguous(), c))
model = MLP_2_Input(B, d, B).to(dev)
fit_probe_to_nearest(model, lambda n, it: (centroid_dist(qb := mq(n, 5000 + it), c, mean, scale), qb), nprobe,
                     steps=100, batch=4096)
pipe = ProbePipeline(idx, c, mean, scale, model, nq, k, 0.5, max_probe=maxp, expect_probes=hint)
pipe.q.copy_(mq(nq, 1335))
for _ in range(reps):
    pipe.run()
torch.cuda.synchronize()
print(cfg, data, "max_probe", maxp, "avg nprobe", pipe.nprobe.float().mean().item())
