import sys, os
sys.path[:0] = [os.path.join(os.getcwd(), "fpn-mt-image-captioning_amd"), os.getcwd()]
import fpnmt, pytest
flag = sys.argv[1] == "on"
fpnmt.config.fuse_residual_grads = flag
print("fuse_residual_grads", flag)
sys.exit(pytest.main(["tests/test_gpu_model.py::test_train_step_parity_c2_model_fp32", "-x", "-q", "-s", "-p", "no:cacheprovider"]))
