"""The synthetic N-sphere generator is deterministic and in the reference schema."""
from raingun_amd.scene import Plane, Sphere
from raingun_amd.synth import SplitMix64, scene_md5, synthetic_scene, synthetic_yaml

# md5 of the YAML the benchmark's 1024-sphere scene is made from (seed 0x5EED)
SYNTH1024_MD5 = "021fa06ed673c2febd5ee6a7df1a00c3"


def test_splitmix64_reference_values():
    r = SplitMix64(0)
    # published SplitMix64 sequence for seed 0
    assert [r.next_u64() for _ in range(3)] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


def test_deterministic():
    assert synthetic_yaml(1024, 2, 5) == synthetic_yaml(1024, 2, 5)
    assert scene_md5(synthetic_yaml(1024, 2, 5)) == SYNTH1024_MD5


def test_shape():
    s = synthetic_scene(4096, 8, 8)
    assert sum(isinstance(b, Sphere) for b in s.bodies) == 4096
    assert sum(isinstance(b, Plane) for b in s.bodies) == 8
    assert s.max_recursion_depth == 8 and len(s.lights) == 3
    kinds = [b.material.surface for b in s.bodies if isinstance(b, Sphere)]
    assert 0.55 < kinds.count("Diffuse") / 4096 < 0.65
    assert 0.12 < kinds.count("Refractive") / 4096 < 0.18
