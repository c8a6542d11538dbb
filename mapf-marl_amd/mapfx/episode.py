"""Device-resident episode storage with the layout and `update` semantics of PyMARL's
EpisodeBatch (MARL-curve-main/src/components/episode_buffer.py:6-134), for runs outside
PyMARL (bench, tests); inside PyMARL the runner is handed the real EpisodeBatch.
Layout: `data.transition_data[key]` = [batch, max_seq_length, *shape], "filled"
added, dtype from the scheme, preprocess outputs (e.g. "actions_onehot") allocated
from each transform's infer_output_info and written by `update` as :128-134;
`update(data, bs, ts, mark_filled)` as :100-134."""
from types import SimpleNamespace as SN

import torch as th


class OneHot:
    """components/transforms.py OneHot (the preprocess PyMARL applies to actions)."""

    def __init__(self, out_dim):
        self.out_dim = out_dim

    def transform(self, tensor):
        y = tensor.new(*tensor.shape[:-1], self.out_dim).zero_()
        y.scatter_(-1, tensor.long(), 1)
        return y.float()

    def infer_output_info(self, vshape_in, dtype_in):
        return (self.out_dim,), th.float32


class DeviceEpisodeBatch:
    def __init__(self, scheme, groups, batch_size, max_seq_length, preprocess=None, device="cpu"):
        self.scheme = dict(scheme)
        self.groups = groups
        self.batch_size = batch_size
        self.max_seq_length = max_seq_length
        self.preprocess = {} if preprocess is None else preprocess
        self.device = device
        self.data = SN(transition_data={}, episode_data={})
        for k, (new_k, transforms) in self.preprocess.items():    # :41-56
            vshape, dtype = self.scheme[k]["vshape"], self.scheme[k].get("dtype", th.float32)
            for tf in transforms:
                vshape, dtype = tf.infer_output_info(vshape, dtype)
            self.scheme[new_k] = {"vshape": vshape, "dtype": dtype}
            if "group" in self.scheme[k]:
                self.scheme[new_k]["group"] = self.scheme[k]["group"]
        self.scheme["filled"] = {"vshape": (1,), "dtype": th.long}
        for k, info in self.scheme.items():
            vshape = info["vshape"]
            vshape = (vshape,) if isinstance(vshape, int) else tuple(vshape)
            group = info.get("group")
            shape = (groups[group], *vshape) if group else vshape
            self.data.transition_data[k] = th.zeros((batch_size, max_seq_length, *shape),
                                                    dtype=info.get("dtype", th.float32),
                                                    device=device)

    def update(self, data, bs=slice(None), ts=slice(None), mark_filled=True):
        if isinstance(bs, list):
            bs = th.as_tensor(bs, dtype=th.long, device=self.device)
        if isinstance(ts, int):
            ts = slice(ts, ts + 1)
        target = self.data.transition_data
        for k, v in data.items():
            if mark_filled:
                target["filled"][bs, ts] = 1
                mark_filled = False
            dtype = self.scheme[k].get("dtype", th.float32)
            v = th.as_tensor(v, device=self.device).to(dtype)
            dest = target[k][bs, ts]
            target[k][bs, ts] = v.reshape(dest.shape)
            if k in self.preprocess:
                new_k, transforms = self.preprocess[k]
                v = target[k][bs, ts]
                for tf in transforms:
                    v = tf.transform(v)
                target[new_k][bs, ts] = v.reshape(target[new_k][bs, ts].shape)

    def __getitem__(self, k):
        return self.data.transition_data[k]
