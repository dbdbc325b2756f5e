"""MI355X-native counterpart of the reference's horovod/mnist_horovod.py (see
pytorch_distributed_examples_amd/apps/mnist_hvd.py for the design notes).

Static:   python -m pytorch_distributed_examples_amd.launch.hvdrun -np 8 horovod_examples/mnist_horovod.py
Torchrun: torchrun --standalone --nproc_per_node 8 horovod_examples/mnist_horovod.py
"""
import os
import sys

if int(os.environ.get("WORLD_SIZE", "1")) > 1:
    os.environ.setdefault("OMP_NUM_THREADS", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_examples_amd.apps.mnist_hvd import main  # noqa: E402

if __name__ == "__main__":
    main()
