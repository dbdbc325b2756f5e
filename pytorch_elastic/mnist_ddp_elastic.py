"""Elastic DDP MNIST training (MI355X-native counterpart of the reference's
pytorch_elastic/mnist_ddp_elastic.py).

Example, 2 nodes x 4 GPUs:
    torchrun --nproc_per_node=4 --nnodes=2 --node_rank=0 --rdzv_id=456 --rdzv_backend=c10d \
        --rdzv_endpoint=<host>:29603 mnist_ddp_elastic.py 10 5
Single node, elastic 2..8 workers, restart on failure:
    torchrun --nnodes=1 --nproc_per_node=8 --rdzv_backend=c10d --rdzv_endpoint=127.0.0.1:29603 \
        --max-restarts=3 mnist_ddp_elastic.py 10 5
"""
import os
import sys

if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # before torch is imported (quirk Q3)
    os.environ.setdefault("OMP_NUM_THREADS", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_examples_amd.apps.mnist_ddp import main  # noqa: E402

if __name__ == "__main__":
    main()
