"""Policy-in-the-loop on the GPU.

`SB2MlpPolicy` is the stable-baselines 2 `FeedForwardPolicy` the reference trained with
PPO2 (trained_model_2v2/model*.zip; colab_notebook.ipynb `PPO2.load(...)`): a tanh MLP
with a shared trunk and separate policy / value heads, the policy head emitting one
logit group per MultiDiscrete sub-action (MultiCategorical).  Deterministic actions
are the per-group argmax (SB2 `predict(obs, deterministic=True)`, which
`evaluate_policy` uses by default).

Weights come from an .npz of the model's `parameters` (tests/golden/extract_sb2_policy.py):
`shared_fc{i}_{w,b}`, `pi_fc{i}_{w,b}`, `vf_fc{i}_{w,b}`, `pi_{w,b}`, `vf_{w,b}`, with
TensorFlow's [in, out] weight layout.  The dense layers run as hipBLASLt GEMMs through
torch on the env's device, fed straight from the env's obs buffer (no host round trip).
"""
import numpy as np
import torch


class SB2MlpPolicy(torch.nn.Module):
    def __init__(self, params, nvec):
        super().__init__()
        self.nvec = [int(n) for n in nvec]

        def stack(prefix):
            layers, i = [], 0
            while "%s%d_w" % (prefix, i) in params:
                layers.append((params["%s%d_w" % (prefix, i)], params["%s%d_b" % (prefix, i)]))
                i += 1
            return layers

        def to_param(w, b):
            return (torch.nn.Parameter(torch.as_tensor(np.ascontiguousarray(w.T)), requires_grad=False),
                    torch.nn.Parameter(torch.as_tensor(b), requires_grad=False))

        self.shared = torch.nn.ParameterList([p for w, b in stack("shared_fc") for p in to_param(w, b)])
        self.pi_net = torch.nn.ParameterList([p for w, b in stack("pi_fc") for p in to_param(w, b)])
        self.vf_net = torch.nn.ParameterList([p for w, b in stack("vf_fc") for p in to_param(w, b)])
        self.pi_w, self.pi_b = to_param(params["pi_w"], params["pi_b"])
        self.vf_w, self.vf_b = to_param(params["vf_w"], params["vf_b"])
        if self.pi_w.shape[0] != sum(self.nvec):
            raise ValueError("policy head has %d logits, action space needs %d" % (self.pi_w.shape[0], sum(self.nvec)))

    @classmethod
    def from_npz(cls, path, nvec, device="cpu"):
        with np.load(path, allow_pickle=False) as z:
            params = {k: z[k] for k in z.files}
        return cls(params, nvec).to(device)

    @staticmethod
    def _mlp(x, plist):
        for i in range(0, len(plist), 2):
            x = torch.tanh(torch.nn.functional.linear(x, plist[i], plist[i + 1]))
        return x

    def forward(self, obs):
        """obs [B, obs_dim] float32 -> (logits [B, sum(nvec)], value [B])."""
        h = self._mlp(obs, self.shared)
        logits = torch.nn.functional.linear(self._mlp(h, self.pi_net), self.pi_w, self.pi_b)
        value = torch.nn.functional.linear(self._mlp(h, self.vf_net), self.vf_w, self.vf_b)[:, 0]
        return logits, value

    @torch.no_grad()
    def act(self, obs, deterministic=True, out=None, generator=None):
        """uint8 actions [B, len(nvec)]: per-group argmax, or a sample of each categorical."""
        logits, _ = self.forward(obs.float())
        groups = torch.split(logits, self.nvec, dim=1)
        if deterministic:
            a = torch.stack([g.argmax(dim=1) for g in groups], dim=1)
        else:
            a = torch.stack([torch.multinomial(torch.softmax(g, dim=1), 1, generator=generator)[:, 0]
                             for g in groups], dim=1)
        if out is None:
            return a.to(torch.uint8)
        out.copy_(a)
        return out
