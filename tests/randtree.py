"""Seeded random URDF trees for property tests (test infrastructure; no reference code)."""
import numpy as np


def random_urdf(rng: np.random.Generator, n_links: int, chain_bias: float = 0.7, box_p: float = 0.3) -> str:
    """A random kinematic tree as URDF text: link 0 is the root; each later link hangs off an earlier one
    (the previous link with probability `chain_bias`, giving long chains); joints are fixed / revolute /
    continuous / prismatic with random origins (xyz + rpy), random or signed axis-aligned axes (some
    unnormalised), and limits; some links carry a box collision."""
    out = ['<robot name="rand">']
    for k in range(n_links):
        out.append(f'  <link name="l{k}">')
        if rng.random() < box_p:
            sx, sy, sz = rng.uniform(0.02, 0.4, 3)
            ox, oy, oz = rng.uniform(-0.1, 0.1, 3)
            r, p, y = rng.uniform(-1, 1, 3)
            out.append(f'    <collision><origin xyz="{ox} {oy} {oz}" rpy="{r} {p} {y}"/>'
                       f'<geometry><box size="{sx} {sy} {sz}"/></geometry></collision>')
        out.append('  </link>')
    for k in range(1, n_links):
        parent = k - 1 if rng.random() < chain_bias else int(rng.integers(0, k))
        jt = rng.choice(["fixed", "revolute", "continuous", "prismatic"], p=[0.2, 0.45, 0.15, 0.2])
        x, y, z = rng.uniform(-0.3, 0.3, 3)
        r, p, yw = rng.uniform(-np.pi, np.pi, 3) * (rng.random() < 0.7)
        s = [f'  <joint name="j{k}" type="{jt}">', f'    <parent link="l{parent}"/>', f'    <child link="l{k}"/>',
             f'    <origin xyz="{x} {y} {z}" rpy="{r} {p} {yw}"/>']
        if jt != "fixed":
            if rng.random() < 0.5:
                a = np.zeros(3)
                a[rng.integers(0, 3)] = rng.choice([-1.0, 1.0])
            else:
                a = rng.normal(size=3)
                if rng.random() < 0.5:
                    a /= np.linalg.norm(a)
            s.append(f'    <axis xyz="{a[0]} {a[1]} {a[2]}"/>')
        if jt == "revolute":
            lo = rng.uniform(-2.5, 0)
            s.append(f'    <limit lower="{lo}" upper="{lo + rng.uniform(0.5, 4)}" effort="1" velocity="1"/>')
        elif jt == "prismatic":
            s.append(f'    <limit lower="{rng.uniform(-0.3, 0)}" upper="{rng.uniform(0.05, 0.4)}" effort="1" velocity="1"/>')
        s.append('  </joint>')
        out += s
    out.append('</robot>')
    return "\n".join(out)
