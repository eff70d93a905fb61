import torch
x = torch.arange(10, dtype=torch.float32, device="cuda")
class B:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 3, "strides": None}
b = B(x.data_ptr(), 10)
try:
    y = torch.as_tensor(b, device="cuda")
    print("as_tensor ok", y.data_ptr() == x.data_ptr(), y[:3].tolist())
except Exception as e:
    print("as_tensor failed", type(e).__name__, e)
try:
    cap = x.__dlpack__()
    z = torch.utils.dlpack.from_dlpack(cap)
    print("dlpack ok", z.data_ptr() == x.data_ptr())
except Exception as e:
    print("dlpack failed", e)
