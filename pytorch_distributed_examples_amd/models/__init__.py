"""Model families: MNIST MLP, MNIST CNN, ResNet-50 pipeline shards, EmbeddingBag hybrid."""
