"""Stride-4 feature encoders used by the Patchifier (reference
dpvo/extractor.py:6-56, 200-264).  Parameter names follow the reference so
its checkpoints load unchanged."""
import torch.nn as nn

BASE = 32


def _norm(kind, ch):
    return {"instance": lambda: nn.InstanceNorm2d(ch), "batch": lambda: nn.BatchNorm2d(ch),
            "group": lambda: nn.GroupNorm(num_groups=ch // 8, num_channels=ch),
            "none": lambda: nn.Sequential()}[kind]()


class ResidualBlock(nn.Module):
    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        self.norm1, self.norm2 = _norm(norm_fn, planes), _norm(norm_fn, planes)
        self.downsample = None
        if stride != 1:
            self.norm3 = _norm(norm_fn, planes)
            self.downsample = nn.Sequential(nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)

    def forward(self, x):
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        return self.relu((x if self.downsample is None else self.downsample(x)) + y)


class BasicEncoder4(nn.Module):
    def __init__(self, output_dim=128, norm_fn="batch", dropout=0.0, multidim=False):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, BASE)
        self.conv1 = nn.Conv2d(3, BASE, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.layer1 = nn.Sequential(ResidualBlock(BASE, BASE, norm_fn, 1), ResidualBlock(BASE, BASE, norm_fn, 1))
        self.layer2 = nn.Sequential(ResidualBlock(BASE, 2 * BASE, norm_fn, 2),
                                    ResidualBlock(2 * BASE, 2 * BASE, norm_fn, 1))
        self.conv2 = nn.Conv2d(2 * BASE, output_dim, kernel_size=1)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def forward(self, x):
        b, n, c, h, w = x.shape
        x = self.relu1(self.norm1(self.conv1(x.view(b * n, c, h, w))))
        x = self.conv2(self.layer2(self.layer1(x)))
        return x.view(b, n, *x.shape[1:])
