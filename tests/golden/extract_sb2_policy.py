"""Extract the trained 2v2 policy weights of the reference (trained_model_2v2/model1.zip,
stable-baselines 2 PPO2) into a plain .npz fixture.  THIS CONTAINER ONLY (the reference does
not travel).  Only the zip's `parameters` member is read, with numpy.load(allow_pickle=False):
it is itself an .npz of float32 arrays.  `data` (cloudpickled policy class) is NOT loaded.

The reference notebook evaluates exactly this model (colab_notebook.ipynb, `PPO2.load(
"trained_model_2v2/model1")`, `evaluate_policy(model, gym.make("Futbol2v2-v1"),
n_eval_episodes=10)`) and prints `mean_reward:2027.02 +/- 1519.25`.
"""
import io
import os
import zipfile

import numpy as np

SRC = "/root/reference/trained_model_2v2/model1.zip"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sb2_2v2_model1.npz")

if __name__ == "__main__":
    with zipfile.ZipFile(SRC) as z:
        p = np.load(io.BytesIO(z.read("parameters")), allow_pickle=False)
        arrays = {k.replace("model/", "").replace(":0", "").replace("/", "_"): p[k] for k in p.files}
    arrays = {k: v for k, v in arrays.items() if not k.startswith("q_")}  # q head: unused by PPO
    np.savez_compressed(DST, **arrays)
    print(DST, {k: v.shape for k, v in arrays.items()})
