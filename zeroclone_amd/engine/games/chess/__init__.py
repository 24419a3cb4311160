"""Chess backend with the reference plugin API (engine/games/chess), rules on the GPU."""
