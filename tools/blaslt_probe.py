import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, itertools
import flexflow_train_amd._ffkernels as k
BF16, F32 = 14, 0   # hipDataType: HIP_R_16BF=14, HIP_R_32F=0
EPI = {"DEFAULT":1, "BIAS":4, "GELU":32, "GELU_BIAS":36, "RELU_AUX_BIAS":134, "GELU_AUX":160, "GELU_AUX_BIAS":164, "DGELU":192, "DGELU_BGRAD":208, "BGRADA":256, "BGRADB":512}
shape=(1024,1024,512)
for name, e in EPI.items():
    for bt in (-1, BF16, F32):
        for at in ((-1, BF16, F32) if "AUX" in name or "DGELU" in name else (-1,)):
            for ta,tb in ((False,False),(True,False),(False,True)):
                for of in (0,1):
                    n = k.blaslt_probe(*shape, ta, tb, e, bt, at, of)
                    if n > 0: print(name, "bias", bt, "aux", at, "ta,tb", ta, tb, "f32out", of, "->", n)
