import ctypes, sys, faulthandler, os
faulthandler.enable()
which = sys.argv[1]
lib_path = sys.argv[2]
if which == "notorch":
    lib = ctypes.CDLL(lib_path)
    print("selftest", lib.diag_selftest(), flush=True)
    sys.exit(0)
import torch
x = torch.zeros(1000, device="cuda")
lib = ctypes.CDLL(lib_path)
if which == "torch_selftest":
    print("selftest", lib.diag_selftest(), flush=True)
    sys.exit(0)
lib.diag_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
print("rc", lib.diag_launch(x.data_ptr(), 1000, torch.cuda.current_stream().cuda_stream), flush=True)
torch.cuda.synchronize()
print("val", x[0].item(), flush=True)
