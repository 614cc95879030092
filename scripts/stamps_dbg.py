import os, sys
os.environ["FUTBOL_LIB_VARIANT"] = "stamps"
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "gym-futbol_amd")]
import torch
from gym_futbol_amd import FutbolVecEnv
B = int(sys.argv[1])
v = FutbolVecEnv("v1", B, device="cuda:0", seed=0, dtype=torch.float32, number_of_player=2)
print("created", flush=True)
v.reset(); torch.cuda.synchronize(); print("reset ok", flush=True)
act = v._act
for t in range(int(sys.argv[2])):
    v.random_actions(2**64 - 1, seed=1234, out=act); torch.cuda.synchronize()
    v.step_raw(act); torch.cuda.synchronize()
    print("step", t, "ok", flush=True)
