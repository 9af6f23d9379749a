"""CPU restatement of ``rl4co/data/transforms.py:15-93`` (test infrastructure only)."""
import math

import torch


def dihedral_8_augmentation(xy):  # transforms.py:15-37
    x, y = xy.split(1, dim=2)
    z = [torch.cat(p, dim=2) for p in ((x, y), (1 - x, y), (x, 1 - y), (1 - x, 1 - y),
                                      (y, x), (1 - y, x), (y, 1 - x), (1 - y, 1 - x))]
    return torch.cat(z, dim=0)


def symmetric_transform(x, y, phi, offset=0.5):  # transforms.py:49-71
    x, y = x - offset, y - offset
    x_prime = torch.cos(phi) * x - torch.sin(phi) * y
    y_prime = torch.sin(phi) * x + torch.cos(phi) * y
    mask = phi > 2 * math.pi
    xy = torch.cat((x_prime, y_prime), dim=-1)
    xy = torch.where(mask, xy.flip(-1), xy)
    return xy + offset
