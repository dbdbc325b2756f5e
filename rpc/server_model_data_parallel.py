"""MI355X-native counterpart of the reference's rpc/server_model_data_parallel.py: parameter server
(EmbeddingBag on "ps") + DDP trainers driven by a master over RPC; `--model resnet50` runs the
BASELINE config-4 hybrid (2-stage pipeline x DDP) under torchrun.
See pytorch_distributed_examples_amd/apps/hybrid_ps.py.

    python rpc/server_model_data_parallel.py [--epochs 100]
    torchrun --standalone --nproc_per_node 8 rpc/server_model_data_parallel.py --model resnet50 --stages 2
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_examples_amd.apps.hybrid_ps import main  # noqa: E402

if __name__ == "__main__":
    main()
