from .ActorCritic import ActorCritic  # noqa: F401
from .RND import RND  # noqa: F401
from .Memory import Memory  # noqa: F401
from .PPO import PPO  # noqa: F401
