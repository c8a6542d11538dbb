"""Device-resident episode storage with the layout and `update` semantics of PyMARL's
EpisodeBatch (MARL-curve-main/src/components/episode_buffer.py:6-134), for runs outside
PyMARL (bench, tests); inside PyMARL the runner is handed the real EpisodeBatch.
Layout: `data.transition_data[key]` = [batch, max_seq_length, *shape], "filled"
added, dtype from the scheme; `update(data, bs, ts, mark_filled)` as :100-134.
Preprocessing transforms are not restated (pass none)."""
from types import SimpleNamespace as SN

import torch as th


class DeviceEpisodeBatch:
    def __init__(self, scheme, groups, batch_size, max_seq_length, preprocess=None, device="cpu"):
        self.scheme = dict(scheme)
        self.groups = groups
        self.batch_size = batch_size
        self.max_seq_length = max_seq_length
        self.device = device
        self.data = SN(transition_data={}, episode_data={})
        scheme = dict(scheme)
        scheme["filled"] = {"vshape": (1,), "dtype": th.long}
        self.scheme["filled"] = scheme["filled"]
        for k, info in scheme.items():
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
        for k, v in data.items():
            target = self.data.transition_data
            if mark_filled:
                target["filled"][bs, ts] = 1
                mark_filled = False
            dtype = self.scheme[k].get("dtype", th.float32)
            v = th.as_tensor(v, device=self.device).to(dtype)
            dest = target[k][bs, ts]
            target[k][bs, ts] = v.reshape(dest.shape)

    def __getitem__(self, k):
        return self.data.transition_data[k]
