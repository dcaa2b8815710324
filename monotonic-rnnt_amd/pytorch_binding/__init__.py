"""PyTorch surface of the MI355X monotonic RNN-T loss (drop-in for the reference's pytorch_binding)."""
from .monotonic_rnnt_joint import MonotonicRNNTJointFunction, monotonic_rnnt_joint_loss
from .monotonic_rnnt_op import MonotonicRNNTFunction, MonotonicRNNTLoss, monotonic_rnnt_cpp, monotonic_rnnt_loss

__all__ = ["MonotonicRNNTFunction", "monotonic_rnnt_loss", "MonotonicRNNTLoss", "monotonic_rnnt_cpp",
           "MonotonicRNNTJointFunction", "monotonic_rnnt_joint_loss"]
