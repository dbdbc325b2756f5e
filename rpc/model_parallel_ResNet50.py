"""MI355X-native counterpart of the reference's rpc/model_parallel_ResNet50.py: a 2-stage ResNet-50
pipeline driven by an RPC master, stages on GPUs, activations GPU->GPU over RCCL.
See pytorch_distributed_examples_amd/apps/resnet_rpc.py.

    python rpc/model_parallel_ResNet50.py [--splits 4 8] [--num-batches 3]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_examples_amd.apps.resnet_rpc import main  # noqa: E402

if __name__ == "__main__":
    main()
