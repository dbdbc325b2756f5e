"""Training applications behind the entry scripts (pytorch_elastic/, horovod/, rpc/)."""
