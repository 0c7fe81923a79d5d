"""``flexflow.torch.fx.torch_to_flexflow`` (the name the reference README
uses, README.md:23-29): trace a module and write its ``.ff`` IR."""
from flexflow_train_amd.frontends.torch_fx import PyTorchModel


def torch_to_flexflow(model, filename):
    PyTorchModel(model).torch_to_file(filename)
