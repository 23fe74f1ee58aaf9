from .tfds import TensorflowDataset
